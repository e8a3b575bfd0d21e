"""Tasks (reference: tasks.py:13-334).

``Task``: dataset registry, ``get_batch_iterator`` (ordered indices ->
native ``batch_by_size`` -> sharded ``EpochBatchIterator``, cached per
dataset), ``train_step`` (``loss = model(*sample)``; ``sample_size =
len(sample[0][0])`` (Q03); ``ntokens = 0`` (Q04)).
``LanguageModelingTask`` (``--task bert``): vocab file, BERT-for-pretraining
from a JSON config, HDF5 shards selected by substring match of the split
name on the full path (Q10), optional ``--num_file`` truncation.
``MNISTTask`` (``--task mnist``): MNISTNet on ``processed/*.pt`` or IDX files.
The reference's broken ``BertFineTuningTask`` (Q13) is replaced by a working
``BertTokenClassificationTask`` built on the same heads.
"""
from __future__ import annotations

import collections
import os

import torch

from hetseq_amd.data import data_utils, iterators
from hetseq_amd.data.mnist_dataset import MNISTDataset, find_split_file, select_split_files


class Task(object):
    def __init__(self, args):
        self.args = args
        self.datasets = {}
        self.dataset_to_epoch_iter = {}

    def load_dictionary(self, vocab_file):
        vocab = collections.OrderedDict()
        index = 0
        with open(vocab_file, "r", encoding="utf-8") as reader:
            while True:
                token = reader.readline()
                if not token:
                    break
                vocab[token.strip()] = index
                index += 1
        print("| loaded dictionary with {} subwords  from: {}".format(index, vocab_file))
        return vocab

    def load_dataset(self, split, **kwargs):
        raise NotImplementedError

    def dataset(self, split):
        if split not in self.datasets:
            raise KeyError("Dataset not loaded: " + split)
        if not isinstance(self.datasets[split], torch.utils.data.Dataset):
            raise TypeError("Datasets are expected to be of type torch.utils.data.Dataset")
        return self.datasets[split]

    def get_batch_iterator(self, dataset, max_tokens=None, max_sentences=None, max_positions=None,
                           ignore_invalid_inputs=False, required_batch_size_multiple=1, seed=1, num_shards=1,
                           shard_id=0, num_workers=0, epoch=0, device=None):
        if dataset in self.dataset_to_epoch_iter:
            return self.dataset_to_epoch_iter[dataset]
        with data_utils.numpy_seed(seed):
            indices = dataset.ordered_indices()
        print("| build batch sampler")
        batch_sampler = data_utils.batch_by_size(indices, dataset.num_tokens, max_tokens=max_tokens,
                                                 max_sentences=max_sentences,
                                                 required_batch_size_multiple=required_batch_size_multiple)
        print("| finish building batch sampler")
        epoch_iter = iterators.EpochBatchIterator(dataset=dataset, collate_fn=dataset.collater,
                                                  batch_sampler=batch_sampler, seed=seed, num_shards=num_shards,
                                                  shard_id=shard_id, num_workers=num_workers, epoch=epoch,
                                                  device=device)
        self.dataset_to_epoch_iter[dataset] = epoch_iter
        return epoch_iter

    def build_model(self, args):
        raise NotImplementedError

    def train_step(self, sample, model, optimizer, ignore_grad=False):
        if not model.training:  # train() walks every submodule: only on a mode change
            model.train()
        loss = model(*sample)
        if ignore_grad:
            loss = loss * 0
        if sample is None or len(sample) == 0 or len(sample[0][0]) == 0:
            sample_size = 0
        else:
            sample_size = len(sample[0][0])
        nsentences = sample_size
        logging_output = {"nsentences": nsentences, "loss": loss.detach(), "nll_loss": loss.detach(), "ntokens": 0,
                          "sample_size": sample_size}
        optimizer.backward(loss)
        return loss, sample_size, logging_output

    def update_step(self, num_updates):
        pass


class LanguageModelingTask(Task):
    """BERT pre-training on NVIDIA-format HDF5 shards."""

    def __init__(self, args, dictionary):
        super().__init__(args)
        self.dictionary = dictionary

    @classmethod
    def setup_task(cls, args, **kwargs):
        dictionary = cls.load_dictionary(cls, args.dict) if getattr(args, "dict", None) else None
        return cls(args, dictionary)

    def build_model(self, args):
        if args.task != "bert":
            raise ValueError("Unsupported language modeling task: {}".format(args.task))
        from hetseq_amd.models.bert import BertConfig, BertForPreTraining

        config = BertConfig.from_json_file(args.config_file)
        model = BertForPreTraining(config)
        return model

    def _split_files(self, split):
        path = self.args.data
        if not os.path.exists(path):
            raise FileNotFoundError("Dataset not found: ({})".format(path))
        files = [os.path.join(path, f) for f in os.listdir(path)] if os.path.isdir(path) else [path]
        files = select_split_files(files, split)
        if self.args.num_file > 0:
            files = files[0:self.args.num_file]
        assert len(files) > 0, "no suitable file in split ***{}***".format(split)
        return files

    def load_dataset(self, split, **kwargs):
        from hetseq_amd.data.bert_dataset import BertH5Dataset, ConBertH5Dataset

        files = self._split_files(split)
        dataset = ConBertH5Dataset([BertH5Dataset(f, self.args.max_pred_length) for f in files])
        print("| loaded {} sentences from: {}".format(len(dataset), self.args.data), flush=True)
        self.datasets[split] = dataset
        print("| loading finished")
        return dataset

    def prepare_model_for_data(self, model, split):
        """Tell the sparse MLM head how many labelled rows a sequence can hold."""
        ds = self.datasets.get(split)
        if ds is not None and hasattr(model, "max_predictions_per_seq"):
            model.max_predictions_per_seq = int(getattr(ds, "num_pred", 0)) or None


class MNISTTask(Task):
    def __init__(self, args):
        super().__init__(args)

    @classmethod
    def setup_task(cls, args, **kwargs):
        return cls(args)

    def build_model(self, args):
        from hetseq_amd.models.mnist import MNISTNet

        return MNISTNet()

    def load_dataset(self, split, **kwargs):
        path = self.args.data
        if not os.path.exists(path):
            raise FileNotFoundError("Dataset not found: ({})".format(path))
        f = find_split_file(path, split if split != "train" else "train")
        dataset = MNISTDataset(f)
        print("| loaded {} sentences from: {}".format(len(dataset), path), flush=True)
        self.datasets[split] = dataset
        print("| loading finished")
        return dataset


class BertTokenClassificationTask(Task):
    """Working replacement for the reference's unreachable BertFineTuningTask (Q13).

    Expects samples ``[input_ids, token_type_ids, attention_mask, labels]``;
    ``args.num_label`` (default 3) labels."""

    def __init__(self, args, dictionary=None):
        super().__init__(args)
        self.dictionary = dictionary

    @classmethod
    def setup_task(cls, args, **kwargs):
        return cls(args, cls.load_dictionary(cls, args.dict) if getattr(args, "dict", None) else None)

    def build_model(self, args):
        from hetseq_amd.models.bert import BertConfig, BertForTokenClassification

        config = BertConfig.from_json_file(args.config_file)
        return BertForTokenClassification(config, getattr(args, "num_label", 3))


def setup_task(args):
    if args.task == "bert":
        return LanguageModelingTask.setup_task(args)
    if args.task == "mnist":
        return MNISTTask.setup_task(args)
    raise ValueError("unsupported task: " + str(args.task))
