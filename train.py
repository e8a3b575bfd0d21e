#!/usr/bin/env python3
"""CLI entry point: ``python train.py [flags]`` (reference: train.py:242).

All flags of the reference are accepted (see hetseq_amd/options.py); the
engine is hetseq_amd (MI355X-native).
"""
from hetseq_amd.train import cli_main

if __name__ == "__main__":
    cli_main()
