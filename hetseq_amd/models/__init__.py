from hetseq_amd.models.bert import (  # noqa: F401
    BertConfig,
    BertForMaskedLM,
    BertForMultipleChoice,
    BertForNextSentencePrediction,
    BertForPreTraining,
    BertForQuestionAnswering,
    BertForSequenceClassification,
    BertForTokenClassification,
    BertModel,
)
from hetseq_amd.models.mnist import MNISTNet  # noqa: F401
