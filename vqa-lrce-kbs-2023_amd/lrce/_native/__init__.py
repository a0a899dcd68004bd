"""ctypes binding of liblrce_hip.so (C ABI declared in include/lrce_hip.h).

The product path calls ONLY these functions for compute; there is no eager/PyTorch fallback.  If
the library (or a GPU) is missing every entry point raises immediately.  Tensors are passed as
raw device pointers; the stream is torch's current HIP stream for the tensor's device.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LRCE_NATIVE_LIB") or os.path.join(_HERE, "liblrce_hip.so")   # override: A/B dev builds

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"liblrce_hip.so not built ({LIB_PATH}); run `python __graft_entry__.py` / make -C csrc")
        L = ctypes.CDLL(LIB_PATH)
        # every entry point declared before the library is handed out: a stale .so missing one raises
        # here on every call, instead of leaving later entries undeclared (ctypes would then pass
        # 64-bit pointers as 32-bit ints into the kernels)
        _declare(L)
        _lib = L
    return _lib


def loaded():
    return _lib is not None


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("a", ctypes.c_void_p), ("b", ctypes.c_void_p), ("c", ctypes.c_void_p),
        ("lda", ctypes.c_int64), ("ldb", ctypes.c_int64), ("ldc", ctypes.c_int64),
        ("stride_a", ctypes.c_int64), ("stride_b", ctypes.c_int64), ("stride_c", ctypes.c_int64),
        ("m", ctypes.c_int32), ("n", ctypes.c_int32), ("k", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("a_kmajor", ctypes.c_int32), ("b_kmajor", ctypes.c_int32), ("a_f32", ctypes.c_int32),
        ("flags", ctypes.c_int32), ("split_k", ctypes.c_int32),
        ("bias", ctypes.c_void_p), ("aux", ctypes.c_void_p), ("ld_aux", ctypes.c_int64),
        ("aux_out", ctypes.c_void_p), ("ld_aux_out", ctypes.c_int64),
        ("a_map", ctypes.c_void_p), ("c_map", ctypes.c_void_p),
        ("alpha", ctypes.c_float), ("scale_cols", ctypes.c_int32), ("scale_val", ctypes.c_float),
        ("row_scale", ctypes.c_void_p), ("rows_per_scale", ctypes.c_int32),
        ("a_row_scale", ctypes.c_void_p), ("a_rows_per_scale", ctypes.c_int32),
        ("b_f32", ctypes.c_int32),
        ("workspace", ctypes.c_void_p), ("workspace_elems", ctypes.c_int64),
        ("drop_p", ctypes.c_float), ("drop_group", ctypes.c_int32), ("drop_seed", ctypes.c_uint64),
        ("f16", ctypes.c_int32), ("alpha_dev", ctypes.c_void_p), ("stride_bias", ctypes.c_int64),
        ("stride_alpha", ctypes.c_int64),
    ]


class MhaDesc(ctypes.Structure):
    _fields_ = [
        ("q", ctypes.c_void_p), ("ld_q", ctypes.c_int64),
        ("k1", ctypes.c_void_p), ("v1", ctypes.c_void_p), ("ld_kv1", ctypes.c_int64), ("stride_kv1_b", ctypes.c_int64),
        ("kv1_bdiv", ctypes.c_int32), ("lk1", ctypes.c_int32),
        ("k2", ctypes.c_void_p), ("v2", ctypes.c_void_p), ("ld_kv2", ctypes.c_int64), ("stride_kv2_b", ctypes.c_int64),
        ("kv2_bdiv", ctypes.c_int32), ("lk2", ctypes.c_int32),
        ("key_mask", ctypes.c_void_p), ("out", ctypes.c_void_p), ("ld_o", ctypes.c_int64), ("lse", ctypes.c_void_p),
        ("B", ctypes.c_int32), ("H", ctypes.c_int32), ("Lq", ctypes.c_int32), ("d", ctypes.c_int32),
        ("scale", ctypes.c_float), ("drop_p", ctypes.c_float), ("seed", ctypes.c_uint64), ("f32_io", ctypes.c_int32),
        ("dout", ctypes.c_void_p), ("dq", ctypes.c_void_p), ("ld_dq", ctypes.c_int64),
        ("dk1", ctypes.c_void_p), ("dv1", ctypes.c_void_p), ("ld_dkv1", ctypes.c_int64), ("stride_dkv1_b", ctypes.c_int64),
        ("dk2", ctypes.c_void_p), ("dv2", ctypes.c_void_p), ("ld_dkv2", ctypes.c_int64), ("stride_dkv2_b", ctypes.c_int64),
        ("f16", ctypes.c_int32), ("dkv1_store", ctypes.c_int32), ("grad16", ctypes.c_int32),
    ]


class LnPrologue(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32), ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("eps", ctypes.c_float),
        ("x", ctypes.c_void_p), ("ld_x", ctypes.c_int64), ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p),
        ("y_out", ctypes.c_void_p), ("ld_y", ctypes.c_int64), ("y2_out", ctypes.c_void_p), ("ld_y2", ctypes.c_int64),
        ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
        ("drop_p", ctypes.c_float), ("drop_group", ctypes.c_int32), ("drop_seed", ctypes.c_uint64),
    ]


class DecKv(ctypes.Structure):
    _fields_ = [
        ("k1", ctypes.c_void_p), ("stride1", ctypes.c_int64), ("ld1", ctypes.c_int64),
        ("bdiv1", ctypes.c_int32), ("lk1", ctypes.c_int32),
        ("k2", ctypes.c_void_p), ("stride2", ctypes.c_int64), ("ld2", ctypes.c_int64),
        ("bdiv2", ctypes.c_int32), ("lk2", ctypes.c_int32), ("v_off", ctypes.c_int64),
    ]


_WS = [("drop_p", ctypes.c_float), ("seed", ctypes.c_uint64), ("slab", ctypes.c_void_p), ("counters", ctypes.c_void_p)]


class DecSa(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("x_in", ctypes.c_void_p), ("ln_gamma", ctypes.c_void_p), ("ln_beta", ctypes.c_void_p),
        ("eps", ctypes.c_float), ("x0_out", ctypes.c_void_p), ("mean_out", ctypes.c_void_p), ("rstd_out", ctypes.c_void_p),
        ("wv", ctypes.c_void_p), ("bv", ctypes.c_void_p), ("wo", ctypes.c_void_p), ("bo", ctypes.c_void_p),
        ("sad", ctypes.c_void_p), ("x1p", ctypes.c_void_p),
    ] + _WS


class DecCa(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("x1p", ctypes.c_void_p), ("g1", ctypes.c_void_p), ("b1", ctypes.c_void_p),
        ("eps", ctypes.c_float), ("x1_out", ctypes.c_void_p), ("mean_out", ctypes.c_void_p), ("rstd_out", ctypes.c_void_p),
        ("wq", ctypes.c_void_p), ("bq", ctypes.c_void_p), ("kv", DecKv), ("q_out", ctypes.c_void_p),
        ("ctx_out", ctypes.c_void_p), ("lse_out", ctypes.c_void_p), ("wo", ctypes.c_void_p), ("bo", ctypes.c_void_p),
        ("x2p", ctypes.c_void_p),
    ] + _WS


class DecCaBwd(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("dx2", ctypes.c_void_p), ("x2p", ctypes.c_void_p), ("mean2", ctypes.c_void_p),
        ("rstd2", ctypes.c_void_p), ("g2", ctypes.c_void_p), ("dcao_out", ctypes.c_void_p), ("wo", ctypes.c_void_p),
        ("kv", DecKv), ("q", ctypes.c_void_p), ("ctx", ctypes.c_void_p), ("lse", ctypes.c_void_p),
        ("dq_out", ctypes.c_void_p), ("dk1", ctypes.c_void_p), ("dstride1", ctypes.c_int64), ("dld1", ctypes.c_int64),
        ("dk2", ctypes.c_void_p), ("dstride2", ctypes.c_int64), ("dld2", ctypes.c_int64), ("dv_off", ctypes.c_int64),
        ("wq", ctypes.c_void_p), ("dx1_out", ctypes.c_void_p),
    ] + _WS + [("dk2_store", ctypes.c_int32), ("dk1_bf16", ctypes.c_void_p)]


class DecSaBwd(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("dx1", ctypes.c_void_p), ("x1p", ctypes.c_void_p), ("mean1", ctypes.c_void_p),
        ("rstd1", ctypes.c_void_p), ("g1", ctypes.c_void_p), ("dsao_out", ctypes.c_void_p), ("wo", ctypes.c_void_p),
        ("dsav_out", ctypes.c_void_p), ("wv", ctypes.c_void_p), ("dx0_out", ctypes.c_void_p),
    ] + _WS


class DecLayerW(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("wv", "bv", "wo", "bo", "g1", "be1", "wq", "bq", "woc", "boc", "g2", "be2",
                                               "w1", "b1", "w2", "b2", "g3", "be3")]


DEC_LAYERS = 12


class DecStep(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("S", ctypes.c_int32), ("step", ctypes.c_int32), ("nmc", ctypes.c_int32),
        ("lt", ctypes.c_int32), ("n_layers", ctypes.c_int32), ("eps", ctypes.c_float), ("drop_p", ctypes.c_float),
        ("seed", ctypes.c_uint64), ("gf", ctypes.c_void_p), ("bf", ctypes.c_void_p),
        ("kv_video", ctypes.c_void_p), ("kv_video_lstride", ctypes.c_int64),
        ("kv_text", ctypes.c_void_p), ("kv_text_lstride", ctypes.c_int64),
        ("acts", ctypes.c_void_p), ("grads", ctypes.c_void_p), ("s_out", ctypes.c_void_p),
        ("ds_in", ctypes.c_void_p), ("ds_out", ctypes.c_void_p),
        ("dkv_video16", ctypes.c_void_p), ("dkv_video32", ctypes.c_void_p), ("dkv_video_lstride", ctypes.c_int64),
        ("dkv_text", ctypes.c_void_p), ("dkv_text_lstride", ctypes.c_int64),
        ("ws", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("status", ctypes.c_void_p),
        ("layer", DecLayerW * DEC_LAYERS),
    ]


class GemmItem(ctypes.Structure):
    _fields_ = [
        ("a", ctypes.c_void_p), ("b", ctypes.c_void_p), ("c", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("alpha_dev", ctypes.c_void_p),
        ("m", ctypes.c_int32), ("n", ctypes.c_int32), ("lda", ctypes.c_int32), ("ldb", ctypes.c_int32),
        ("ldc", ctypes.c_int32), ("flags", ctypes.c_int32), ("f16", ctypes.c_int32),
        ("split", ctypes.c_int32), ("k_chunk", ctypes.c_int32),
    ]


class SlabSum(ctypes.Structure):
    _fields_ = [("slabs", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("split", ctypes.c_int32), ("accumulate", ctypes.c_int32)]


EPI_BIAS, EPI_GELU, EPI_DGELU, EPI_RESID = 1, 2, 4, 8
EPI_OUT_F32, EPI_ATOMIC, EPI_ACCUM, EPI_AUX_OUT, EPI_OUT_BOTH = 16, 32, 64, 128, 256
EPI_BIAS_GRAD = 512
EPI_SLABS = 1024
EPI_AUX_F32 = 2048

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float
_U64 = ctypes.c_uint64

_SIGS = {
    "lrce_gemm": [ctypes.POINTER(GemmDesc), _P],
    "lrce_gemm_ln": [ctypes.POINTER(GemmDesc), ctypes.POINTER(LnPrologue), _P],
    "lrce_gemm_ptr_batched": [ctypes.POINTER(GemmDesc), _P, _P, _P, _P, _I, _P],
    "lrce_gemm_grouped": [ctypes.POINTER(GemmItem), _I, _I, _F, _P],
    "lrce_slab_sum_grouped": [ctypes.POINTER(SlabSum), _I, _P],
    "lrce_splitk_reduce_ln": [_P, _I, _I, _I, _P, _P, _I64, _F, _U64, _P, _P, _P, _F, _P, _P, _I, _P, _P, _P],
    "lrce_layernorm_fwd": [_P, _I, _P, _I, _P, _P, _F, _P, _I, _P, _P, _P, _P, _I, _I, _I, _P],
    "lrce_layernorm_bwd": [_P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P, _I64,
                           _P],
    "lrce_scale_cast_bf16": [_P, _I64, _I, _P, _I, _P, _P],
    "lrce_wattn_bias_build": [_P, _P, _I, _I, _I, _P, _I, _P, _I, _P, _I, _P],
    "lrce_wattn_fwd_grouped": [_P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _P],
    "lrce_wattn_qkv_fwd": [_P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "lrce_wattn_bwd": [_P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "lrce_wattn_dbias": [_P, _I, _I, _I, _P, _P, _P],
    "lrce_wattn_dbias_batched": [_P, _P, _P, _P, _P, _P, _I, _P],
    "lrce_layernorm_bwd_deferred": [_P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P,
                                    _I64, _P, _P],
    "lrce_layernorm_grad_reduce": [_P, _P, _P, _P, _P, _I, _P],
    "lrce_layernorm_bwd_f16s_deferred": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _F, _U64, _P, _I64, _P, _P],
    "lrce_mha_fwd": [ctypes.POINTER(MhaDesc), _P],
    "lrce_mha_bwd": [ctypes.POINTER(MhaDesc), _P],
    "lrce_dec_sa_fwd": [ctypes.POINTER(DecSa), _P],
    "lrce_dec_ca_fwd": [ctypes.POINTER(DecCa), _P],
    "lrce_dec_ca_bwd": [ctypes.POINTER(DecCaBwd), _P],
    "lrce_dec_sa_bwd": [ctypes.POINTER(DecSaBwd), _P],
    "lrce_dec_ln_grads": [_P, _P, _P, _P, _P, _P, _I, _I, _P],
    "lrce_dec_set_trace": [_P],
    "lrce_dec_step_fwd": [ctypes.POINTER(DecStep), _P],
    "lrce_dec_step_bwd": [ctypes.POINTER(DecStep), _P],
    "lrce_dec_step_reset": [_P, _P, _P, _P],
    "lrce_dec_step_field": [_I, _I, _I, _I, _I, _I],
    "lrce_dec_step_ws_elems": [],
    "lrce_dec_step_counter_words": [],
    "lrce_dec_step_grid": [_I],
    "lrce_dec_step_set_trace": [_P],
    "lrce_wattn_set_trace": [_P],
    "lrce_gemm_set_trace": [_P],
    "lrce_frames_resize": [_P, _I, _I, _I, _P, _I, _I, _I, _P, _P],
    "lrce_patch_im2col": [_P, _I, _I, _I, _I, _I64, _I64, _I64, _I, _P, _P],
    "lrce_colsum": [_P, _I, _P, _I64, _I, _I, _P, _I, _P, _P],
    "lrce_cast_bf16": [_P, _P, _I64, _P],
    "lrce_sum_shards_bf16": [_P, _I, _I64, _P, _P],
    "lrce_cast_f16": [_P, _P, _I64, _P],
    "lrce_cast_f16_bf16": [_P, _P, _I64, _P],
    "lrce_dropout": [_P, _P, _P, _P, _I64, _F, _U64, _I64, _P],
    "lrce_dropout_bwd": [_P, _P, _P, _I64, _F, _U64, _I64, _P],
    "lrce_grad_scale": [_P, _I64, _P, _P],
    "lrce_grad_scale_update": [_P, _I, _P],
    "lrce_layernorm_bwd_f16s": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _F, _U64, _P, _I64, _P],
    "lrce_dropout_bwd_f16": [_P, _P, _I64, _F, _U64, _I64, _P, _P],
    "lrce_bert_embed_fwd": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "lrce_bert_embed_bwd": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I64, _P],
    "lrce_video_posembed_fwd": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "lrce_video_posembed_bwd": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "lrce_text_posembed_fwd": [_P, _P, _P, _P, _I, _I, _I, _P],
    "lrce_text_posembed_bwd": [_P, _P, _P, _P, _I, _I, _I, _P],
    "lrce_l2norm_multi": [_P, _P, _I, _P, _I, _P, _P, _P],
    "lrce_adamw_step": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _F, _F, _F, _F, _F, _P, _P, _P, _I64, _I64,
                        _P, _P, _P, _I, _P, _I, _I64, _I64, _P],
    "lrce_set_rng_offset": [_P],
    "lrce_version": [],
    "lrce_last_error": [],
}
_RET = {"lrce_last_error": ctypes.c_char_p, "lrce_wattn_bias_elems": _I64, "lrce_wattn_dbias_part_elems": _I64,
        "lrce_layernorm_bwd_workspace": _I64}
_SIGS["lrce_wattn_bias_elems"] = [_I, _I]
_SIGS["lrce_dec_slab_elems"] = [_I]
_RET["lrce_dec_slab_elems"] = _I64
_SIGS["lrce_wattn_dbias_part_elems"] = [_I, _I, _I]
_RET.update({"lrce_dec_step_field": _I64, "lrce_dec_step_ws_elems": _I64, "lrce_dec_step_counter_words": _I64})
_SIGS["lrce_layernorm_bwd_workspace"] = [_I, _I]


def _declare(L):
    missing = [name for name in _SIGS if not hasattr(L, name)]
    if missing:
        raise NativeError(f"{LIB_PATH} lacks {missing[:5]} ({len(missing)} entry points): a stale build — "
                          "rebuild with `python __graft_entry__.py`")
    for name, args in _SIGS.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = _RET.get(name, ctypes.c_int)


def exported_symbols():
    return sorted(_SIGS)


def ptr(t):
    return None if t is None else t.data_ptr()


def stream_of(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def call(name, *args):
    if torch._C._autograd._profiler_enabled():
        # visible in torch.profiler traces as lrce::<entry point> (the launch itself is async)
        with torch.profiler.record_function("lrce::" + name[5:]):
            rc = getattr(lib(), name)(*args)
    else:
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed ({rc}): {lib().lrce_last_error().decode()}")
