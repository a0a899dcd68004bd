#!/usr/bin/env python
"""train.py — LRCE training with args.py's flags (temporal scale default [1, 2, 3], validation on the
'val' split); same data-parallel driver as train_ddp.py (reference train.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lrce import cli  # noqa: E402

if __name__ == "__main__":
    cli.launch(cli.train_main, cli.parse_arg_train(temporal_default=(1, 2, 3)), "val")
