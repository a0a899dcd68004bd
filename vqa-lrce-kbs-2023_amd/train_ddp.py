#!/usr/bin/env python
"""train_ddp.py — data-parallel LRCE training (reference train_ddp.py; flags of parser.py).
    python train_ddp.py --dataset msvd-qa-oe --synthetic 200 --batch-size 10 --epoch 1 --debug-mode
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_ddp.py --dataset msrvtt-qa-oe --synthetic 800 ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lrce import cli  # noqa: E402

if __name__ == "__main__":
    cli.launch(cli.train_main, cli.parse_arg_train(temporal_default=(3,)), "test")
