"""Synthetic stand-in for the reference E2E datasets (lrce/dataset/e2e_dataset.py).

Video decoding, annotation files and the WordPiece tokenizer are out of scope (SURVEY §8 f, rank 2);
this dataset yields items with exactly the reference's item contract (e2e_dataset.py:118-124,
164-182, 219-317) so the agents, DistributedSampler and DataLoader run unchanged:

    video_clips       (sum(temporal_scale), frames_per_clip, 3, 224, 224) f32 in [0, 1)
                      -- the multi-scale sampling result of e2e_dataset.py:96-116 (scale s adds s clips)
    input_ids         (L,) int64  (OE / count)  |  (5, L) int64 (MC)
    attention_mask    same shape, 1 on real tokens
    token_type_ids    same shape, 0 on the question, 1 on the answer part (MC, e2e_dataset.py:219-295)
    ground_truth      () int64 answer index, IGNORE_INDEX (-100) for out-of-vocabulary answers in OE
                      (e2e_dataset.py:182); () int64 choice index (MC); () f32 count (count task)

Questions are "[CLS] q_1..q_{n} [SEP] <pad>" with n = question_tokens - 2 WordPiece ids drawn from
[1000, 30522); MC rows append "a_1..a_m [SEP]" (type id 1).  Every item is a pure function of
(seed, index), so every rank / epoch sees the same data for the same index.
"""
import torch

IGNORE_INDEX = -100
CLS_ID, SEP_ID = 101, 102


class SyntheticQADataset(torch.utils.data.Dataset):
    def __init__(self, size, task_type="oe", max_text_token_len=32, temporal_scale=(3,), frames_per_clip=5,
                 num_classes=1000, question_tokens=20, answer_tokens=4, total_mc=5, resolution=224,
                 ignore_fraction=0.0, seed=0):
        if task_type not in ("oe", "mc", "count"):
            raise ValueError(f"unsupported task type {task_type!r}")
        if question_tokens + (answer_tokens + 1 if task_type == "mc" else 0) > max_text_token_len:
            raise ValueError("question (+ answer) does not fit max_text_token_len")
        self.size = int(size)
        self.task_type = task_type
        self.seq_len = int(max_text_token_len)
        self.n_clips = int(sum(temporal_scale))
        self.frames = int(frames_per_clip)
        self.num_classes = int(num_classes)
        self.q_tokens = int(question_tokens)
        self.a_tokens = int(answer_tokens)
        self.total_mc = int(total_mc)
        self.res = int(resolution)
        self.ignore_fraction = float(ignore_fraction)
        self.seed = int(seed)

    def __len__(self):
        return self.size

    def _gen(self, idx):
        return torch.Generator().manual_seed(self.seed * 1_000_003 + idx)

    def _question(self, g):
        ids = torch.zeros(self.seq_len, dtype=torch.int64)
        n = self.q_tokens
        ids[0], ids[n - 1] = CLS_ID, SEP_ID
        ids[1:n - 1] = torch.randint(1000, 30522, (n - 2,), generator=g)
        return ids, n

    def __getitem__(self, idx):
        if not 0 <= idx < self.size:
            raise IndexError(idx)
        g = self._gen(idx)
        clips = torch.rand(self.n_clips, self.frames, 3, self.res, self.res, generator=g)
        if self.task_type == "mc":
            ids = torch.zeros(self.total_mc, self.seq_len, dtype=torch.int64)
            types = torch.zeros_like(ids)
            q, n = self._question(g)
            for c in range(self.total_mc):
                ids[c] = q
                a = self.a_tokens
                ids[c, n:n + a] = torch.randint(1000, 30522, (a,), generator=g)
                ids[c, n + a] = SEP_ID
                types[c, n:n + a + 1] = 1
            mask = (ids != 0).long()
            gt = torch.randint(0, self.total_mc, (), generator=g)
            return clips, ids, mask, types, gt
        ids, _ = self._question(g)
        mask = (ids != 0).long()
        types = torch.zeros_like(ids)
        if self.task_type == "count":
            gt = torch.randint(1, 11, (), generator=g).float()
            return clips, ids, mask, types, gt
        gt = torch.randint(0, self.num_classes, (), generator=g)
        if self.ignore_fraction > 0 and torch.rand((), generator=g).item() < self.ignore_fraction:
            gt = torch.tensor(IGNORE_INDEX)
        return clips, ids, mask, types, gt
