#!/usr/bin/env python3
"""MNIST evaluator (reference: eval_mnist.py:39-100).

Loads ``checkpoint['model']`` into MNISTNet and reports average loss and
accuracy on the test split.  The checkpoint is read with
``weights_only=True`` (argparse.Namespace allow-listed).
"""
import argparse

import torch

from hetseq_amd.checkpoint_utils import load_checkpoint_to_cpu
from hetseq_amd.data.mnist_dataset import MNISTDataset, find_split_file
from hetseq_amd.models.mnist import MNISTNet


def main(argv=None):
    parser = argparse.ArgumentParser(description="evaluate a trained MNIST checkpoint")
    parser.add_argument("--model_ckpt", "--model-ckpt", required=True, type=str)
    parser.add_argument("--mnist_dir", "--mnist-dir", required=True, type=str)
    parser.add_argument("--batch-size", default=64, type=int)
    parser.add_argument("--cpu", action="store_true")
    args = parser.parse_args(argv)
    device = torch.device("cuda" if torch.cuda.is_available() and not args.cpu else "cpu")
    state = load_checkpoint_to_cpu(args.model_ckpt)
    model = MNISTNet()
    model.load_state_dict(state["model"])
    model.to(device).eval()
    ds = MNISTDataset(find_split_file(args.mnist_dir, "test"))
    loader = torch.utils.data.DataLoader(ds, batch_size=args.batch_size, shuffle=False, collate_fn=ds.collater)
    test_loss, correct = 0.0, 0
    with torch.no_grad():
        for x, y in loader:
            loss, c = model(x.to(device), y.to(device), eval=True)
            test_loss += float(loss)
            correct += int(c)
    test_loss /= len(ds)
    acc = 100.0 * correct / len(ds)
    print("\nTest set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n".format(test_loss, correct, len(ds), acc))
    return test_loss, acc


if __name__ == "__main__":
    main()
