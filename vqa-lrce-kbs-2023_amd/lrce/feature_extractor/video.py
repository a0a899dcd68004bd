"""VideoExtractor (reference lrce/feature_extractor/video.py:6-43) on the native Swin3D.

Differences from the reference, all behaviour-preserving:
* the S temporal-scale clips are processed as ONE Swin batch of B*S clips instead of S sequential
  calls (video.py:33-40) — per-clip math is independent, so outputs are identical;
* ImageNet Normalize (video.py:35) and the T padding are fused into the patch-embed im2col kernel;
* the Kinetics-600 checkpoint (`state_dict` keys `backbone.*`, video.py:20-26) is loaded when the
  file exists (weights_only).  The reference asserts it exists (e2e.py:11); here a missing file
  leaves the random initialisation with a warning and `pretrained_loaded = False`, and the training
  CLI refuses to start from it unless the run is synthetic or --allow-random-init is given
  (lrce/cli.py) — a real run cannot silently train from a random backbone.  ckpt_path=None: random
  initialisation on purpose (tests, benchmarks), no warning.
"""
import os
import warnings
from collections import OrderedDict

import torch
import torch.nn as nn

from .video_swin import SwinTransformer3D

SWIN_B_CKPT = "./pretrained_models/swin_base_patch244_window877_kinetics600_22k.pth"


class VideoExtractor(nn.Module):
    def __init__(self, ckpt_path=None):
        super().__init__()
        self.swin = SwinTransformer3D(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                                      patch_size=(2, 4, 4), window_size=(8, 7, 7), drop_path_rate=0.2,
                                      patch_norm=True)
        self.pretrained_loaded = False
        if ckpt_path and os.path.exists(ckpt_path) and os.path.getsize(ckpt_path) > 0:
            ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
            sd = OrderedDict((k[9:], v) for k, v in ckpt["state_dict"].items() if "backbone" in k)
            self.swin.load_state_dict(sd)
            self.pretrained_loaded = True
        elif ckpt_path:
            warnings.warn(f"Swin checkpoint {ckpt_path} not found: the video backbone keeps its random "
                          "initialisation", stacklevel=2)

    def forward(self, clips):
        """clips (B, S, T, 3, H, W) f32 in [0,1] -> (B, S, (T+1)//2, (H//32)*(W//32), 1024)."""
        B, S = clips.shape[:2]
        feats, (nc, D, h, w) = self.swin.forward_tokens(clips.contiguous())
        return feats.view(B, S, D, h * w, feats.shape[-1])
