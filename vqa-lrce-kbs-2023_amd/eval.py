#!/usr/bin/env python
"""eval.py — evaluate a `{'model_state_dict': ...}` checkpoint (reference eval.py; flags of
args.py:parse_arg_eval).
    python eval.py --dataset msvd-qa-oe --model-path runs/<uid>_msvd-qa-oe/weights/best.pt --synthetic 40
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lrce import cli  # noqa: E402

if __name__ == "__main__":
    cli.launch(cli.eval_main, cli.parse_arg_eval())
