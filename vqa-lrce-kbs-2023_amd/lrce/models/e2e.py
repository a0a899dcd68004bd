"""End-to-end LRCE models (reference lrce/models/e2e.py) on the gfx950 path.

Same classes, constructor signatures (positional as train_ddp.py:89-98, keyword as eval.py:66-74),
attributes (`text_extractor`, `video_extractor`, `fusion_model`) and forward contract:
    forward(video_clips (B,S,T,3,H,W) f32, texts (B,L)|(B,5,L) int64, texts_attention_mask,
            texts_type_ids) -> (B,num_classes) | (B,5) | (B,)
The reference asserts the Kinetics-600 Swin checkpoint exists (e2e.py:11) and downloads BERT by
name (text.py:9); this build loads the Swin checkpoint and a local BERT copy when present (keyword
arguments swin_ckpt / bert_dir; None = random initialisation on purpose), warns otherwise, never
touches the network, and exposes `pretrained_loaded` so the training CLI can refuse a real run that
would start from random backbones.
"""
from typing import Iterable, List

import torch
import torch.nn as nn

from ..feature_extractor.text import TextExtractor, BERT_DIR
from ..feature_extractor.video import VideoExtractor, SWIN_B_CKPT
from .. import kernels as K
from ..runtime import prepare, side_stream
from .fusionv3 import LRCEOpenEnded, LRCEMultipleChoice, LRCECount


def _head_args(feature_dim, num_classes, drop_out_rate, video_feature_res, video_feature_dim, frame_sample_size,
               temporal_scale, text_seq_len):
    """The positional argument list every LRCE head takes (fusionv3.py:137-151)."""
    return (feature_dim, num_classes, drop_out_rate, video_feature_res, video_feature_dim, frame_sample_size,
            temporal_scale, text_seq_len)


class E2EBase(nn.Module):
    """Swin3D video extractor + BERT text extractor + an LRCE head (HEAD, set by the subclasses);
    forward(clips, texts, mask, types) -> head(video features, text features, mask)."""
    HEAD = None

    def __init__(self, *head_args, swin_ckpt=SWIN_B_CKPT, bert_dir=BERT_DIR) -> None:
        super().__init__()
        # split backward (data-parallel graph mode, lrce/graph.TrainStepGraph(tail=...)): the fusion
        # head runs on leaf copies of the extractor features, so loss.backward() stops at them and
        # backward_extractors() continues from their gradients — the gradient exchange of the head's
        # buckets overlaps the extractors' backward between the two captured graphs
        self.split_backward = False
        self._split = None
        # with split_backward, also cut the Swin backward before this stage (None: one segment): the
        # buckets of the stages above it (stages 3-4 of Swin-B: ~82 M of its 87.6 M parameters) and
        # of BERT are exchanged while the stages below replay (backward_segments)
        self.split_swin_stage = None
        self.text_extractor = TextExtractor(bert_dir=bert_dir)
        self.video_extractor = VideoExtractor(swin_ckpt)
        if self.HEAD is not None:
            self.fusion_model = self.HEAD(*_head_args(*head_args))

    def extract_text_features(self, texts, attention_mask, texts_type_ids, join_token=None):
        return self.text_extractor(texts, attention_mask, texts_type_ids, join_token=join_token)

    @property
    def pretrained_loaded(self):
        """Both backbones came from checkpoints (Swin Kinetics-600 + BERT)."""
        return self.video_extractor.pretrained_loaded and self.text_extractor.pretrained_loaded

    def lrce_param_order(self):
        """Flat-store layout = reverse forward order (fusion, BERT top-down, Swin top-down), so the
        gradient buckets complete in sequence during backward; the unused BERT pooler goes last."""
        fusion = list(self.fusion_model.parameters())[::-1]
        bert = self.text_extractor.bert
        pool = {id(p) for p in bert.pooler.parameters()}
        text = [p for p in self.text_extractor.parameters() if id(p) not in pool][::-1]
        video = list(self.video_extractor.parameters())[::-1]
        return fusion + text + video + list(bert.pooler.parameters())

    def optimizer_groups(self):
        """Parameter groups whose gradients are final before the whole backward is (FusedAdamW
        .enable_early_updates): the recurrent decoder (its backward ends before the extractors'),
        the BERT encoder (its backward runs on the side stream beside Swin's), and Swin stages 4, 3,
        2 (the backward runs stage 4 -> 1; stage 4's group carries the final LayerNorm)."""
        pool = {id(p) for p in self.text_extractor.bert.pooler.parameters()}
        swin = self.video_extractor.swin
        text = [p for p in self.text_extractor.parameters() if id(p) not in pool]
        groups = {"decoder": list(self.fusion_model.fusion_transformer.parameters()), "text": text}
        for i in range(len(swin.layers) - 1, 0, -1):
            ps = list(swin.layers[i].parameters())
            if i == len(swin.layers) - 1:
                ps += list(swin.norm.parameters())
            groups[swin.layers[i].blocks[0]._lrce_group] = ps
        return groups

    def overflow_guard(self, device):
        """(parameters, scale slots) for FusedAdamW's found-inf guard: BERT's backward runs on fp16
        operands with delayed per-tensor scales (text.py), and an operand that overflowed raises its
        slot's flag; the text group (the parameters those operands' gradients reach) then keeps its
        values for the step, as the reference's GradScaler skips an overflowing step (agent_oe.py:40-42)."""
        pool = {id(p) for p in self.text_extractor.bert.pooler.parameters()}
        text = [p for p in self.text_extractor.parameters() if id(p) not in pool]
        return text, self.text_extractor.bert._grad_scales(torch.device(device))

    def extract_video_features(self, video_clips):
        return self.video_extractor(video_clips)

    def forward(self, video_clips, texts, texts_attention_mask, texts_type_ids):
        """The two extractors are independent until the fusion head: BERT runs on a side stream
        while Swin runs on the current one (forward and, through autograd's stream semantics,
        backward); a leaf join token consumed by the text branch makes autograd join the side stream
        back at the end of backward, and the fusion head waits for the text features."""
        flat = prepare(self)
        if self.training:
            K.rng_advance(flat.device)   # fresh dropout masks per step, also under HIP-graph replay
            if torch.is_grad_enabled():
                flat.step_begin()        # optimizer step bookkeeping, before any stream forks
        main = torch.cuda.current_stream(flat.device)
        side = side_stream(flat.device)
        tok = None
        if torch.is_grad_enabled():
            tok = getattr(self, "_join_token", None)
            if tok is None or tok.device != flat.device:
                tok = torch.zeros(1, device=flat.device, requires_grad=True)
                object.__setattr__(self, "_join_token", tok)
        side.wait_stream(main)
        swin = self.video_extractor.swin
        swin.split_at = self.split_swin_stage if self.split_backward else None
        with torch.cuda.stream(side):
            t = self.extract_text_features(texts, texts_attention_mask, texts_type_ids, join_token=tok)
        v = self.extract_video_features(video_clips)
        main.wait_stream(side)
        t.record_stream(main)
        if self.split_backward and torch.is_grad_enabled():
            v_in, t_in = v.detach().requires_grad_(True), t.detach().requires_grad_(True)
            self._split = (v, t, v_in, t_in)
            return self.fusion_model(v_in, t_in, texts_attention_mask)
        return self.fusion_model(v, t, texts_attention_mask)

    def backward_extractors(self):
        """Second half of a split backward: the extractors' backward (Swin on this stream, BERT on its
        side stream, joined at the end) from the feature gradients loss.backward() left."""
        self._backward_upper()
        if self.video_extractor.swin._split_mid is not None:
            self.video_extractor.swin.backward_below_split()

    def _backward_upper(self):
        v, t, v_in, t_in = self._split
        self._split = None
        torch.autograd.backward([v, t], [v_in.grad, t_in.grad])

    def backward_segments(self):
        """The extractors' backward as TrainStepGraph tail segments: one, or two when split_swin_stage
        cuts the Swin backward — [BERT + Swin stages >= split_swin_stage, the stages below it + the
        patch embedding]."""
        if self.split_swin_stage is None:
            return [self.backward_extractors]
        return [self._backward_upper, self.video_extractor.swin.backward_below_split]


# Constructor defaults differ per task (question length 30 vs 40, one output for counting), so each
# class restates the signature (positional order of train_ddp.py:89-98, keywords of eval.py:66-74).
class E2EOpenEnded(E2EBase):
    HEAD = LRCEOpenEnded

    def __init__(self, feature_dim: int, num_classes: int, drop_out_rate: float = 0.1,
                 video_feature_res: Iterable[int] = (7, 7), video_feature_dim: int = 768, frame_sample_size: int = 5,
                 temporal_scale: List[int] = [1, 2, 3], text_seq_len: int = 30, **pretrained) -> None:
        super().__init__(feature_dim, num_classes, drop_out_rate, video_feature_res, video_feature_dim,
                         frame_sample_size, temporal_scale, text_seq_len, **pretrained)


class E2EMultipleChoice(E2EBase):
    HEAD = LRCEMultipleChoice

    def __init__(self, feature_dim: int, num_classes: int, drop_out_rate: float = 0.1,
                 video_feature_res: Iterable[int] = (7, 7), video_feature_dim: int = 768, frame_sample_size: int = 5,
                 temporal_scale: List[int] = [1, 2, 3], text_seq_len: int = 40, **pretrained) -> None:
        super().__init__(feature_dim, num_classes, drop_out_rate, video_feature_res, video_feature_dim,
                         frame_sample_size, temporal_scale, text_seq_len, **pretrained)

    def extract_text_features(self, texts, attention_mask, texts_type_ids, join_token=None):
        """e2e.py:77-81: the 5 question+answer sequences go through BERT as B*5 rows."""
        b, n_choice, seq = texts.shape
        feats = self.text_extractor(texts.flatten(0, 1), attention_mask.flatten(0, 1), texts_type_ids.flatten(0, 1),
                                    join_token=join_token)
        return feats.view(b, n_choice, seq, -1)


class E2ECount(E2EBase):
    HEAD = LRCECount

    def __init__(self, feature_dim: int, num_classes: int = 1, drop_out_rate: float = 0.1,
                 video_feature_res: Iterable[int] = (7, 7), video_feature_dim: int = 768, frame_sample_size: int = 5,
                 temporal_scale: List[int] = [1, 2, 3], text_seq_len: int = 30, **pretrained) -> None:
        super().__init__(feature_dim, num_classes, drop_out_rate, video_feature_res, video_feature_dim,
                         frame_sample_size, temporal_scale, text_seq_len, **pretrained)



