from hetseq_amd.optim.lr_scheduler import PolynomialDecayScheduler, build_lr_scheduler  # noqa: F401
from hetseq_amd.optim.optimizers import _Adadelta, _Adam, _Lamb, _Optimizer, build_optimizer  # noqa: F401
