"""ctypes binding of libsdiar.so (include/sdiar.h).

The HIP library is the only compute path: if it is missing or fails to load,
every entry point raises immediately — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDIAR_LIB", os.path.join(_HERE, "lib", "libsdiar.so"))

SD_OK = 0
SD_ERR_INVALID = -1
SD_ERR_SHAPE = -2
SD_ERR_PARAM = -3
SD_ERR_HIP = -4
SD_ERR_STATE = -5


class SdiarError(RuntimeError):
    """Device / runtime failure inside libsdiar."""


class TsvadConfig(ctypes.Structure):
    _fields_ = [
        ("variant", c_int),
        ("max_num_speaker", c_int),
        ("rs_len", c_int),
        ("max_batch", c_int),
        ("max_fbank_frames", c_int),
        ("precision", c_int),
        ("num_transformer_layer", c_int),
        ("num_attention_head", c_int),
        ("transformer_embed_dim", c_int),
        ("transformer_ffn_embed_dim", c_int),
        ("speaker_embed_dim", c_int),
    ]


class EdaConfig(ctypes.Structure):
    _fields_ = [
        ("variant", c_int),
        ("in_size", c_int),
        ("n_units", c_int),
        ("n_heads", c_int),
        ("n_layers", c_int),
        ("dim_feedforward", c_int),
        ("max_seqs", c_int),
        ("max_frames", c_int),
        ("max_n_speakers", c_int),
        ("precision", c_int),
        ("n_speakers", c_int),
    ]


class FseendConfig(ctypes.Structure):
    _fields_ = [
        ("in_size", c_int),
        ("n_units", c_int),
        ("n_heads", c_int),
        ("enc_n_layers", c_int),
        ("enc_dim_feedforward", c_int),
        ("dec_n_layers", c_int),
        ("dec_dim_feedforward", c_int),
        ("conv_delay", c_int),
        ("mask_delay", c_int),
        ("has_mask", c_int),
        ("max_seqs", c_int),
        ("max_frames", c_int),
        ("max_nspks", c_int),
        ("precision", c_int),
    ]


class CamppConfig(ctypes.Structure):
    _fields_ = [
        ("feat_dim", c_int),
        ("embedding_size", c_int),
        ("max_batch", c_int),
        ("max_frames", c_int),
        ("precision", c_int),
    ]


class SsndConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "max_batch", "max_fbank_frames", "max_speakers", "feat_dim", "emb_dim", "q_det_aux_dim", "q_rep_aux_dim",
        "d_model", "nhead", "d_ff", "num_layers", "vad_out_len", "pos_emb_dim", "max_seq_len", "n_all_speakers",
        "conformer_kernel", "precision")]


class TsvadStreamConfig(ctypes.Structure):
    _fields_ = [
        ("max_num_speaker", c_int),
        ("max_labels", c_int),
        ("precision", c_int),
        ("num_transformer_layer", c_int),
        ("num_attention_head", c_int),
        ("transformer_embed_dim", c_int),
        ("transformer_ffn_embed_dim", c_int),
        ("speaker_embed_dim", c_int),
        ("max_windows", c_int),
    ]


_SIGS = {
    "sd_last_error": (c_char_p, []),
    "sd_version": (c_int, []),
    "sd_prof_enable": (None, [c_int]),
    "sd_prof_reset": (None, []),
    "sd_prof_query": (c_int, [c_int, c_char_p, c_int, POINTER(c_int64), POINTER(ctypes.c_double),
                              POINTER(ctypes.c_double), POINTER(ctypes.c_double)]),
    "sd_prof_query_steps": (ctypes.c_double, [c_int]),
    "sd_probe_lstm_granule2": (c_int, [c_int, c_void_p, c_void_p]),
    "sd_probe_lstm_granule": (c_int, [c_int, c_void_p, c_void_p]),
    "sd_probe_lstm_handoff": (c_int, [c_int, c_void_p, c_void_p]),
    "sd_tsvad_create": (c_int, [POINTER(TsvadConfig), POINTER(c_void_p)]),
    "sd_tsvad_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_tsvad_finalize": (c_int, [c_void_p]),
    "sd_tsvad_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "sd_tsvad_status": (c_int, [c_void_p, c_void_p]),
    "sd_tsvad_forward_batched": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                         c_void_p]),
    "sd_tsvad_forward_graph": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_char_p,
                                       c_void_p]),
    "sd_tsvad_debug_buffer": (c_int, [c_void_p, c_int, POINTER(c_void_p), POINTER(c_int64)]),
    "sd_tsvad_device_bytes": (c_int64, [c_void_p]),
    "sd_tsvad_destroy": (c_int, [c_void_p]),
    "sd_tsvad_stream_create": (c_int, [POINTER(TsvadStreamConfig), POINTER(c_void_p)]),
    "sd_tsvad_stream_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_tsvad_stream_finalize": (c_int, [c_void_p]),
    "sd_tsvad_stream_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                        c_void_p]),
    "sd_tsvad_stream_device_bytes": (c_int64, [c_void_p]),
    "sd_tsvad_stream_destroy": (c_int, [c_void_p]),
    "sd_ssnd_create": (c_int, [POINTER(SsndConfig), POINTER(c_void_p)]),
    "sd_ssnd_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_ssnd_finalize": (c_int, [c_void_p]),
    "sd_ssnd_infer": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sd_ssnd_decode": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sd_ssnd_device_bytes": (c_int64, [c_void_p]),
    "sd_ssnd_destroy": (c_int, [c_void_p]),
    "sd_campp_create": (c_int, [POINTER(CamppConfig), POINTER(c_void_p)]),
    "sd_campp_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_campp_finalize": (c_int, [c_void_p]),
    "sd_campp_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sd_campp_device_bytes": (c_int64, [c_void_p]),
    "sd_campp_destroy": (c_int, [c_void_p]),
    "sd_eda_create": (c_int, [POINTER(EdaConfig), POINTER(c_void_p)]),
    "sd_eda_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_eda_finalize": (c_int, [c_void_p]),
    "sd_eda_input_stride": (c_int, [c_void_p]),
    "sd_eda_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "sd_eda_status": (c_int, [c_void_p, c_void_p]),
    "sd_eda_device_bytes": (c_int64, [c_void_p]),
    "sd_eda_destroy": (c_int, [c_void_p]),
    "sd_fseend_create": (c_int, [POINTER(FseendConfig), POINTER(c_void_p)]),
    "sd_fseend_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "sd_fseend_finalize": (c_int, [c_void_p]),
    "sd_fseend_input_stride": (c_int, [c_void_p]),
    "sd_fseend_test": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "sd_fseend_device_bytes": (c_int64, [c_void_p]),
    "sd_fseend_destroy": (c_int, [c_void_p]),
    "sd_fseend_stream_create": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "sd_fseend_stream_push": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, POINTER(c_int), c_void_p]),
    "sd_fseend_stream_set_audio": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int]),
    "sd_fseend_stream_push_audio": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int, POINTER(c_int), c_void_p]),
    "sd_fseend_stream_flush": (c_int, [c_void_p, c_void_p, c_int, POINTER(c_int), c_void_p]),
    "sd_fseend_stream_reset": (c_int, [c_void_p, c_void_p]),
    "sd_fseend_stream_device_bytes": (c_int64, [c_void_p]),
    "sd_fseend_stream_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int), POINTER(c_int)]),
    "sd_fseend_stream_debug_counters": (c_int, [c_void_p, POINTER(ctypes.c_uint), c_int, POINTER(c_int), c_void_p]),
    "sd_fseend_stream_destroy": (c_int, [c_void_p]),
    "sd_eend_features": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                 c_void_p, c_void_p, c_int, c_void_p]),
    "sd_fbank_kaldi": (c_int, [c_void_p, c_int64, c_float, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "sd_fbank_kaldi_ex": (c_int, [c_void_p, c_int64, c_float, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sd_window_cmn": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sd_overlap_average": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                   c_void_p, c_void_p]),
    "sd_overlap_mean": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                c_void_p, c_void_p]),
    "sd_postprocess_segments": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                        c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "sd_op_add_layernorm": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_int,
                                    c_void_p, c_int, c_void_p]),
    "sd_op_linear": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    "sd_op_gemm_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "sd_debug_cam_dense_probe": (c_int, [c_void_p]),
    "sd_debug_rowprog_probe": (c_int, [c_void_p]),
    "sd_probe_graph_memset": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p]),
    "sd_op_mha_block": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "sd_op_cam_dense": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_int, c_void_p]),
    "sd_op_conv1d": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_void_p, c_int, c_void_p]),
    "sd_op_conv2d": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "sd_op_attention": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                c_void_p]),
    "sd_op_attention_grid": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                     c_void_p]),
    "sd_op_attention_chunk": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                      c_void_p]),
    "sd_probe_attention_mask": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                        c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "sd_op_layernorm": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p]),
    "sd_op_lstm": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """Load libsdiar.so (raises if it is missing: the product has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsdiar.so not found at {LIB_PATH}; build it with "
            "`python -m speaker_diarization_amd.build` (HIP extension is required)")
    lib = ctypes.CDLL(LIB_PATH)
    # SDIAR_LIB (A/B runs against an older build) may lack entry points added since; the in-tree build
    # must export every one of them
    ab = os.environ.get("SDIAR_LIB") is not None
    for name, (res, args) in _SIGS.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str = ""):
    if status == SD_OK:
        return
    msg = load().sd_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if status == SD_ERR_INVALID:
        raise ValueError(msg)
    if status == SD_ERR_SHAPE:
        raise AssertionError(msg)
    if status == SD_ERR_PARAM:
        raise RuntimeError(f"Error(s) in loading state_dict: {msg}")
    raise SdiarError(msg)


def has(name: str) -> bool:
    """Whether the loaded library exports `name` (only an older SDIAR_LIB build in an A/B run may not)."""
    return hasattr(load(), name)


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)


def create_handle(kind: str, conf, state) -> ctypes.c_void_p:
    """sd_<kind>_create + set_param for every state_dict entry (reference key names)
    + finalize; the handle is destroyed again if any step fails."""
    import numpy as np
    lib = load()
    h = ctypes.c_void_p()
    call(f"sd_{kind}_create", ctypes.byref(conf), ctypes.byref(h))
    try:
        for k, v in state.items():
            a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
            shape = (c_int64 * max(a.ndim, 1))(*a.shape)
            call(f"sd_{kind}_set_param", h, k.encode(), a.ctypes.data_as(c_void_p), shape, a.ndim)
        call(f"sd_{kind}_finalize", h)
    except Exception:
        getattr(lib, f"sd_{kind}_destroy")(h)
        raise
    return h


def host_state(state_dict) -> dict:
    """state_dict (torch tensors or arrays) -> {key: float32 numpy} on the host."""
    import numpy as np
    return {k: (v.detach().cpu().float().numpy() if hasattr(v, "detach") else np.asarray(v, dtype=np.float32))
            for k, v in state_dict.items()}


def ptr(t) -> int:
    """Raw device/host pointer of a contiguous torch tensor (None -> NULL)."""
    if t is None:
        return None
    assert t.is_contiguous(), "sdiar expects contiguous tensors"
    return t.data_ptr()


def prof_stats():
    """{family: dict(launches, flops, bytes, ms)} from the library's event timers."""
    lib = load()
    out = {}
    i = 0
    buf = ctypes.create_string_buffer(128)
    while True:
        l, f, b, ms = c_int64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        if not lib.sd_prof_query(i, buf, 128, ctypes.byref(l), ctypes.byref(f), ctypes.byref(b), ctypes.byref(ms)):
            break
        steps = lib.sd_prof_query_steps(i) if hasattr(lib, "sd_prof_query_steps") else 0.0
        out[buf.value.decode()] = dict(launches=l.value, flops=f.value, bytes=b.value, ms=ms.value, steps=steps)
        i += 1
    return out


def stream_ptr(device=None):
    import torch
    return torch.cuda.current_stream(device).cuda_stream
