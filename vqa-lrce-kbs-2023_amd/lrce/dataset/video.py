"""Video clip assembly on the device (reference lrce/dataset/e2e_dataset.py:36-116).

The reference decodes a whole video with cv2 on the CPU, resizes EVERY frame to 224x224 through
PIL + torchvision (Resize + ToTensor), then keeps only the frames its multi-scale rule selects.
Here the rule runs first on frame indices (host integer arithmetic, identical slicing), and only
the selected frames are resampled — on the GPU, by one kernel that restates Pillow's antialiased
BILINEAR resample bit for bit (csrc/video_io.hip) and writes the (clips, frames, 3, 224, 224)
layout the video extractor consumes.  Decoding itself (cv2.VideoCapture) stays with the caller:
it hands over decoded RGB frames as uint8 [T, H, W, 3].
"""
import torch

from .. import kernels as K

# e2e_dataset.py:36-45: rows of a pre-extracted (.npy) multi-scale clip stack used per temporal scale
# (scale 4 starts at row 5, overlapping scale 3's last row, exactly as in the reference)
EXTRACTED_SCALE_ROWS = {1: [0], 2: [1, 2], 3: [3, 4, 5], 4: [5, 6, 7, 8]}


def extracted_scale_index(temporal_scale):
    """e2e_dataset.py:_build_scale_idx: row indices of a pre-extracted clip stack."""
    idx = []
    for scale in temporal_scale:
        idx += EXTRACTED_SCALE_ROWS[scale]
    return idx


def multiscale_frame_indices(total_frames, frames_per_clip=5, temporal_scale=(1, 2, 3)):
    """Frame indices of e2e_dataset.py:_get_video_clips (:86-111), clip-major: for each scale s,
    frames are strided by max(1, max(1, T // fpc) // s) starting at half a stride, and s clips of fpc
    consecutive strided frames start inner_step apart.  Raises like the reference's assertions."""
    if total_frames < frames_per_clip:
        raise ValueError(f"video has {total_frames} frames < frames_per_clip {frames_per_clip}")
    frames = list(range(total_frames))
    out = []
    for scale in temporal_scale:
        step = max(1, max(1, total_frames // frames_per_clip) // scale)
        strided = frames[step // 2::step]
        inner = (len(strided) - frames_per_clip) // (scale - 1) if scale > 1 else 0
        for i in range(scale):
            clip = strided[i * inner:i * inner + frames_per_clip]
            if len(clip) != frames_per_clip:
                raise ValueError(f"Mismatch length of clips in scale {scale}: expected {frames_per_clip}, got {len(clip)}")
            out += clip
    return out


def clips_from_frames(frames, frames_per_clip=5, temporal_scale=(1, 2, 3), frame_size=(224, 224), out=None):
    """Decoded RGB frames uint8 [T, H, W, 3] on the GPU -> video_clips f32 [S, fpc, 3, h, w] in [0, 1]
    (S = sum(temporal_scale)), the reference dataset item's first element."""
    if frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError("frames must be uint8 [T, H, W, 3]")
    idx = multiscale_frame_indices(frames.shape[0], frames_per_clip, temporal_scale)
    idx_t = torch.tensor(idx, dtype=torch.int32).to(frames.device, non_blocking=True)
    h, w = frame_size
    res = K.frames_resize(frames, idx_t, h, w, out=out)
    return res.view(len(idx) // frames_per_clip, frames_per_clip, 3, h, w)
