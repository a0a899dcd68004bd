"""Stand-in modules that let the read-only reference (/root/reference) be imported in THIS
container to generate golden vectors.  Only used by tests/golden/make_golden.py — never on the
GPU box, never by the product.

The reference imports several packages that are absent here (cv2, h5py, torchvision, timm,
mmcv, tensorboard, cosine_annealing_warmup).  None of them contributes arithmetic to the hot path
except:
  * torchvision.transforms.Normalize  (video.py:35)  -> (x - mean_c) / std_c on dim -3
  * timm DropPath (identity in eval)    (video_swin_ori.py:11, 243)
  * timm trunc_normal_                  (init only; overwritten by our weight recipe)
These are restated below with the published semantics of torchvision 0.13 / timm 0.4.12.
"""
import sys
import types

import torch


def _mod(name):
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


def install():
    if "torchvision" in sys.modules and getattr(sys.modules["torchvision"], "_lrce_stub", False):
        return
    # transformers must be imported before a fake torchvision exists (it probes torchvision).
    import transformers  # noqa: F401

    _mod("cv2")
    _mod("h5py")

    tv = _mod("torchvision")
    tv._lrce_stub = True
    tvt = _mod("torchvision.transforms")
    tv.transforms = tvt

    class Normalize:
        def __init__(self, mean, std):
            self.mean = torch.tensor(mean, dtype=torch.float32)
            self.std = torch.tensor(std, dtype=torch.float32)

        def __call__(self, x):
            m = self.mean.to(x.device, x.dtype).view(-1, 1, 1)
            s = self.std.to(x.device, x.dtype).view(-1, 1, 1)
            return (x - m) / s

    tvt.Normalize = Normalize

    timm = _mod("timm")
    tm = _mod("timm.models")
    tml = _mod("timm.models.layers")
    timm.models = tm
    tm.layers = tml

    class DropPath(torch.nn.Module):
        def __init__(self, drop_prob=None):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1 - self.drop_prob
            shape = (x.shape[0],) + (1,) * (x.ndim - 1)
            r = keep + torch.rand(shape, dtype=x.dtype, device=x.device)
            r.floor_()
            return x.div(keep) * r

    tml.DropPath = DropPath
    tml.trunc_normal_ = lambda t, mean=0.0, std=1.0, a=-2.0, b=2.0: torch.nn.init.trunc_normal_(t, mean, std, a, b)

    mmcv = _mod("mmcv")
    mu = _mod("mmcv.utils")
    mr = _mod("mmcv.runner")
    mmcv.utils = mu
    mmcv.runner = mr
    mu.get_logger = lambda *a, **k: None
    mr.load_checkpoint = lambda *a, **k: None

    tb = _mod("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

    tb.SummaryWriter = SummaryWriter
    caw = _mod("cosine_annealing_warmup")
    caw.CosineAnnealingWarmupRestarts = object

    if "/root/reference" not in sys.path:
        sys.path.insert(0, "/root/reference")
