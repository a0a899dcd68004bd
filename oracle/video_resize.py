"""CPU restatement (TEST INFRASTRUCTURE ONLY — the checker, never the product path) of the clip
assembly of the reference dataset (lrce/dataset/e2e_dataset.py:60-111): torchvision
Resize((h, w)) on a PIL image = Pillow's antialiased BILINEAR resample (third-party: Pillow,
Resample.c precompute_coeffs / normalize_coeffs_8bpc / ImagingResample{Horizontal,Vertical}_8bpc;
the reference pins no Pillow version — pinned here to Pillow 12.2.0's own output by
tests/golden/frames_resize.npz), then ToTensor (/255), and the multi-scale frame selection.
"""
import numpy as np

PREC = 22   # PRECISION_BITS = 32 - 8 - 2


def _coeffs(in_size, out_size):
    """Fixed-point tap matrix [out_size, in_size] (int64) of Pillow's bilinear filter."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = fs
    K = np.zeros((out_size, in_size), dtype=np.int64)
    for i in range(out_size):
        center = (i + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) / fs)) for x in range(xmax)]
        ww = sum(w)
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            K[i, xmin + x] = int(-0.5 + k * (1 << PREC)) if k < 0 else int(0.5 + k * (1 << PREC))
    return K


def _clip8(v):
    return np.clip(v >> PREC, 0, 255)


def pil_bilinear_resize(img, out_h, out_w):
    """uint8 [H, W, 3] -> uint8 [out_h, out_w, 3], Pillow Image.resize((out_w, out_h), BILINEAR)."""
    x = img.astype(np.int64)
    H, W, _ = x.shape
    if out_w != W:
        x = _clip8(np.einsum("ow,hwc->hoc", _coeffs(W, out_w), x) + (1 << (PREC - 1)))
    if out_h != H:
        x = _clip8(np.einsum("oh,hwc->owc", _coeffs(H, out_h), x) + (1 << (PREC - 1)))
    return x.astype(np.uint8)


def multiscale_frame_indices(total_frames, frames_per_clip, temporal_scale):
    """e2e_dataset.py:96-111 on frame indices (the reference slices the decoded-frame tensor)."""
    assert total_frames >= frames_per_clip
    frames = list(range(total_frames))
    out = []
    for scale in temporal_scale:
        step_size = max(1, max(1, len(frames) // frames_per_clip) // scale)
        scale_res_all = frames[step_size // 2::step_size]
        inner_step_size = (len(scale_res_all) - frames_per_clip) // (scale - 1) if scale > 1 else 0
        for i in range(scale):
            clips = scale_res_all[i * inner_step_size:i * inner_step_size + frames_per_clip]
            assert len(clips) == frames_per_clip
            out += clips
    return out
