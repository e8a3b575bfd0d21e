from hetseq_amd.data import data_utils, iterators  # noqa: F401
from hetseq_amd.data.mnist_dataset import MNISTDataset  # noqa: F401


def __getattr__(name):
    # the HDF5 dataset needs the native _h5 module; import it lazily
    if name in ("BertH5Dataset", "ConBertH5Dataset", "NativeBatchStream"):
        from hetseq_amd.data import bert_dataset

        return getattr(bert_dataset, name)
    raise AttributeError(name)
