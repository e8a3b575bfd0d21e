"""MNIST CNN (reference: tasks.py:337-362, eval_mnist.py:9-37).

conv(1->32,3) -> ReLU -> conv(32->64,3) -> ReLU -> maxpool2 -> Dropout2d(.25)
-> flatten -> fc(9216->128) -> ReLU -> Dropout2d(.5) -> fc(128->10) ->
log_softmax -> NLL.  ``forward(x, target)`` returns the loss (task contract);
``eval=True`` returns (loss summed over the batch, number correct) for the
evaluator.  On a GPU the whole network runs on the gfx950 kernels of
``ops/mnist_ops.py`` (K15); ``logits`` is the torch-op path (CPU, and the
numerics oracle of tests/test_mnist_gpu.py).
"""
import torch
import torch.nn.functional as F
from torch import nn


class MNISTNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout2d(0.25)
        self.dropout2 = nn.Dropout2d(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def logits(self, x):
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        # reference applies Dropout2d to [N, 128]; under torch 1.6 every (n, c) is a
        # 1-element "channel", i.e. element-wise dropout -- reproduce that directly
        x = F.dropout(x, p=self.dropout2.p, training=self.training)
        return self.fc2(x)

    def forward(self, x, target, eval=False):
        from hetseq_amd.ops._C import use_fused

        if use_fused(x) and x.shape[1:] == (1, 28, 28):  # K15: the whole network on the gfx950 kernels
            from hetseq_amd.ops.mnist_ops import mnist_loss

            loss, correct = mnist_loss(self, x, target, eval=eval)
            return (loss, correct) if eval else loss
        output = F.log_softmax(self.logits(x), dim=1)
        if eval:
            loss = F.nll_loss(output, target, reduction="sum")
            correct = output.argmax(dim=1).eq(target).sum()
            return loss, correct
        return F.nll_loss(output, target)
