"""ctypes binding of libcai.so (the C ABI declared in include/cai.h).

The product path has no fallback: if the library is missing or a call fails
the error is raised (ValueError for argument/shape errors, RuntimeError for
device errors), mirroring the reference's ``std::domain_error -> ValueError``
convention (cpp_exts/ops/ops.cpp:46-64).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("CAI_LIB", os.path.join(_PKG_ROOT, "lib", "libcai.so"))

CAI_OK, CAI_EINVAL, CAI_EDEVICE, CAI_EWORKSPACE = 0, 1, 2, 3
F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2
MASK_NONE, MASK_POS, MASK_LEAKY, MASK_SIGN = 0, 1, 2, 3
MASK_BEFORE_RES = 16   # flag: the dgrad mask scales the conv's input gradient only (cai.h CAI_MASK_BEFORE_RES)
Q_NOISE, Q_DEQUANTIZE, Q_SYMBOLS = 0, 1, 2
ADAM_CLIP, ADAM_SKIP_NONFINITE, ADAM_ZERO_GRAD = 1, 2, 4          # cai_adam_step flags (include/cai.h)
ADAM_SMALL_N = 1 << 16                         # cai_adam_step: one-block path at or below this many parameters


class ConvGeom(Structure):
    _fields_ = [(n, c_int32) for n in (
        "batch", "in_c", "in_h", "in_w", "out_c", "out_h", "out_w",
        "kernel", "stride", "pad", "output_padding", "transposed")]


class WindowAttn(Structure):
    _fields_ = [("q", c_void_p), ("q_ld", c_int32), ("kv", c_void_p), ("kv_ld", c_int32), ("bias_table", c_void_p),
                ("rel_index", c_void_p), ("mask", c_void_p), ("B", c_int32), ("Hr", c_int32), ("Wr", c_int32),
                ("heads", c_int32), ("head_dim", c_int32), ("window", c_int32), ("shift", c_int32),
                ("scale", c_float)]


NOISE_BUF, NOISE_DRAW, NOISE_REPLAY = 0, 1, 2             # cai_noise_src kinds (include/cai.h)
NOISE_STATE_WORDS = 144                                  # CAI_NOISE_STATE_WORDS


class NoiseSrc(Structure):
    _fields_ = [("kind", c_int32), ("ld", c_int32), ("buf", c_void_p), ("state", c_void_p), ("slot", c_void_p)]


class EbParams(Structure):
    _fields_ = [("matrix", c_void_p * 5), ("bias", c_void_p * 5), ("factor", c_void_p * 4), ("quantiles", c_void_p)]


class RdInputs(Structure):
    _fields_ = [("lik", c_void_p * 4), ("lik_n", c_int64 * 4), ("nlik", c_int32), ("x_hat", c_void_p),
                ("target", c_void_p), ("n", c_int64)]


class RdGrads(Structure):
    _fields_ = [("dlik", c_void_p * 4)]


class EbGrads(Structure):
    _fields_ = [("matrix", c_void_p * 5), ("bias", c_void_p * 5), ("factor", c_void_p * 4), ("quantiles", c_void_p),
                ("accumulate", c_int32)]


JOB_NONE, JOB_WGRAD, JOB_GDN, JOB_EDGE = 0, 1, 2, 3           # cai_reduce_job kinds (include/cai.h)
GC_SCALES_RELU = 16                                              # cai_gc_bwd mode flag


class ReduceJob(Structure):
    _fields_ = [("kind", c_int32), ("nblocks", c_int32), ("i", c_int32 * 10), ("f", c_float * 2), ("p", c_void_p * 6)]


class WgradCall(Structure):
    """cai_wgrad_call: one weight-gradient call of cai_conv_wgrad_batch."""
    _fields_ = [("geom", ConvGeom), ("dtype", c_int32), ("x", c_void_p), ("x_ld", c_int32), ("in_abs", c_int32),
                ("in_sq", c_int32), ("dy", c_void_p), ("dy_ld", c_int32), ("dw", c_void_p), ("db", c_void_p),
                ("accumulate", c_int32), ("workspace", c_void_p), ("ws_bytes", c_size_t)]


class ResunitArgs(Structure):
    _fields_ = [("batch", c_int32), ("h", c_int32), ("w", c_int32), ("n", c_int32),
                ("x", c_void_p), ("y", c_void_p), ("wa", c_void_p), ("wb", c_void_p), ("wc", c_void_p),
                ("ba", c_void_p), ("bb", c_void_p), ("bc", c_void_p), ("h1", c_void_p), ("h2", c_void_p),
                ("out", c_void_p), ("gc", c_void_p), ("gb", c_void_p), ("ga", c_void_p), ("res2", c_void_p),
                ("xmask", c_void_p), ("x_ld", c_int32), ("y_ld", c_int32), ("out_ld", c_int32),
                ("res2_ld", c_int32), ("xmask_ld", c_int32), ("kpa", c_int32), ("kpb", c_int32), ("kpc", c_int32),
                ("gy_masked", c_int32)]


class ResunitWgradArgs(Structure):
    _fields_ = [("batch", c_int32), ("h", c_int32), ("w", c_int32), ("n", c_int32),
                ("x", c_void_p), ("h1", c_void_p), ("h2", c_void_p), ("ga", c_void_p), ("gb", c_void_p),
                ("gc", c_void_p), ("x_ld", c_int32), ("gc_ld", c_int32), ("dwa", c_void_p), ("dba", c_void_p),
                ("dwb", c_void_p), ("dbb", c_void_p), ("dwc", c_void_p), ("dbc", c_void_p), ("accumulate", c_int32)]


# name -> (restype, argtypes)
_P, _I, _I64, _F, _S = c_void_p, c_int, c_int64, c_float, c_size_t
_G = POINTER(ConvGeom)
_N = POINTER(NoiseSrc)
SIGNATURES = {
    "cai_last_error": (c_char_p, []),
    "cai_version": (c_int, []),
    "cai_abi_count": (c_int, []),
    "cai_conv_packed_weight_bytes": (_S, [_G, _I, _I]),
    "cai_conv_pack_weight": (_I, [_G, _I, _I, _P, _P, _P, _P]),
    "cai_conv_pack_desc_bytes": (_S, []),
    "cai_conv_pack_describe": (_I, [_G, _I, _I, _P, _P, _P, _P]),
    "cai_conv_pack_finalize": (_I64, [_P, c_int32]),
    "cai_conv_pack_many": (_I, [_P, c_int32, _I, _I64, _P]),
    "cai_pack_nchw": (_I, [_P, c_int32, c_int32, c_int32, c_int32, _I, _P, c_int32, _P]),
    "cai_conv_workspace_bytes": (_S, [_G, _I, _I]),
    "cai_conv_fwd": (_I, [_G, _I, _P, c_int32, c_int32, _P, _P, c_int32, _F, _P, _I, _I64, _I64, _I64, _I64,
                          _P, _S, _P]),
    "cai_conv_fwd_res": (_I, [_G, _I, _P, c_int32, c_int32, _P, _P, c_int32, _F, _P, c_int32, _P, _I, _I64, _I64,
                              _I64, _I64, _P, _S, _P]),
    "cai_conv_dgrad": (_I, [_G, _I, _P, c_int32, _P, _P, c_int32, c_int32, _F, _P, c_int32, _P, _S, _P]),
    "cai_conv_dgrad_res": (_I, [_G, _I, _P, c_int32, _P, _P, c_int32, _P, c_int32, c_int32, _F, _P, c_int32, _P, _S,
                                _P]),
    "cai_conv_dgrad_res2": (_I, [_G, _I, _P, c_int32, _P, _P, c_int32, _P, c_int32, _P, c_int32, c_int32, _F, _P,
                                 c_int32, _P, _S, _P]),
    "cai_conv_wgrad_workspace_bytes": (_S, [_G, _I]),
    "cai_resunit": (_I, [POINTER(ResunitArgs), c_int32, _P]),
    "cai_resunit_wgrad_workspace_bytes": (_S, [POINTER(ResunitWgradArgs)]),
    "cai_resunit_wgrad": (_I, [POINTER(ResunitWgradArgs), _P, _S, _P, POINTER(ReduceJob)]),
    "cai_conv_kernel_name": (c_char_p, [_G, _I, _I, c_int32]),
    "cai_conv_split_factor": (c_int32, [_G, _I, _I, c_int32]),
    "cai_conv_wgrad": (_I, [_G, _I, _P, c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, _S, _P]),
    "cai_conv_wgrad_deferred": (_I, [_G, _I, _P, c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, _S, _P,
                                     POINTER(ReduceJob)]),
    "cai_reduce_jobs": (_I, [POINTER(ReduceJob), c_int32, _P]),
    "cai_reduce_jobs_grid": (_I, [POINTER(ReduceJob), c_int32, c_int32, _P]),
    "cai_conv_wgrad_batch": (_I, [POINTER(WgradCall), c_int32, _P, POINTER(ReduceJob)]),
    "cai_resunit_wgrad_batch": (_I, [POINTER(ResunitWgradArgs), POINTER(c_void_p), POINTER(c_size_t), c_int32, _P,
                                    POINTER(ReduceJob)]),
    "cai_deconv_small_workspace_bytes": (_S, [_G, _I]),
    "cai_deconv_small_fwd": (_I, [_G, _I, _P, c_int32, _P, _P, _P, _P, _S, _P]),
    "cai_deconv_small_bwd": (_I, [_G, _I, _P, c_int32, _P, _P, _P, c_int32, _P, _P, c_int32, _P, _S, _P]),
    "cai_edge_supported": (_I, [_G, _I]),
    "cai_edge_workspace_bytes": (_S, [_G, _I]),
    "cai_edge_frag_bytes": (_S, [_G, _I, _I]),
    "cai_edge_pack_weights": (_I, [_G, _I, _I, _P, _P, _P]),
    "cai_edge_pack_describe": (_I, [_G, _I, _I, _P, _P, _P]),
    "cai_edge_conv_fwd": (_I, [_G, _P, _P, _P, _P, c_int32, _P]),
    "cai_edge_deconv_fwd": (_I, [_G, _P, c_int32, _P, _P, _P, _P]),
    "cai_edge_deconv_dgrad": (_I, [_G, _P, _P, _P, c_int32, _P]),
    "cai_edge_wgrad": (_I, [_G, _P, _P, c_int32, _P, _P, c_int32, _P, _S, _P]),
    "cai_edge_wgrad_deferred": (_I, [_G, _P, _P, c_int32, _P, _P, c_int32, _P, _S, _P, POINTER(ReduceJob)]),
    "cai_add_act": (_I, [_I, _P, c_int32, _P, c_int32, _P, c_int32, _I64, c_int32, c_int32, _F, _P]),
    "cai_axpy_dev": (_I, [_I64, _P, _P, _P, _P]),
    "cai_act": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, c_int32, _F, _P]),
    "cai_gdn1_out": (_I, [_I, _P, c_int32, _P, c_int32, _P, c_int32, _I64, c_int32, c_int32, _P]),
    "cai_gdn1_out_bwd": (_I, [_I, _P, c_int32, _P, c_int32, _P, c_int32, _P, c_int32, _P, c_int32, _I64, c_int32,
                              c_int32, _P]),
    "cai_gate_fwd": (_I, [_I, _P, _P, _P, _P, c_int32, _I64, c_int32, _P]),
    "cai_gate_bwd": (_I, [_I, _P, _P, _P, c_int32, _P, _P, c_int32, _I64, c_int32, c_int32, _P]),
    "cai_pixel_shuffle": (_I, [_I, _P, POINTER(c_int64), _P, POINTER(c_int64), c_int32, c_int32, c_int32, c_int32,
                               c_int32, c_int32, _P]),
    "cai_layernorm_fwd": (_I, [_I, _P, c_int32, _I64, c_int32, _P, _P, _F, _P, c_int32, _P, _P, _P]),
    "cai_layernorm_bwd_workspace_bytes": (_S, [_I64, c_int32]),
    "cai_layernorm_bwd": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, _P, _P, _P, _P, c_int32, _P, _P, c_int32,
                               _P, _S, _P]),
    "cai_gelu_fwd": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, _P]),
    "cai_gelu_bwd": (_I, [_I, _P, c_int32, _P, c_int32, _P, c_int32, _I64, c_int32, _P]),
    "cai_window_attn_fwd": (_I, [_I, POINTER(WindowAttn), _P, c_int32, _P]),
    "cai_window_attn_bwd_workspace_bytes": (_S, [POINTER(WindowAttn)]),
    "cai_window_attn_bwd": (_I, [_I, POINTER(WindowAttn), _P, c_int32, _P, c_int32, _P, c_int32, _P, c_int32, _P, _S,
                                 _P]),
    "cai_channel_mean_workspace_bytes": (_S, [c_int32, _I64, c_int32]),
    "cai_channel_mean": (_I, [_I, _P, c_int32, _P, c_int32, c_int32, _I64, c_int32, _P, _F, _P, _S, _P]),
    "cai_channel_affine": (_I, [_I, _P, c_int32, _P, _P, _F, _P, c_int32, c_int32, _I64, c_int32, _P]),
    "cai_gdn_reparam": (_I, [_P, _P, c_int32, _F, _F, _I, _P, _P, _P]),
    "cai_gdn_reparam_describe": (_I, [_P, _P, c_int32, _F, _F, _P, _P, _P]),
    "cai_gdn_fwd": (_I, [_I, _P, c_int32, _I64, c_int32, _P, _P, c_int32, _P, c_int32, _P]),
    "cai_gdn_bwd": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, _P, _P, c_int32, _P, c_int32, _P, _P]),
    "cai_gdn_param_grad_workspace_bytes": (_S, [_I64, c_int32, _I]),
    "cai_gdn_param_grad": (_I, [_I, _P, c_int32, _P, _I64, c_int32, _P, _P, _F, _F, _P, _P, c_int32, _P, _S, _P]),
    "cai_gdn_backward_workspace_bytes": (_S, [_I64, c_int32, _I]),
    "cai_gdn_kernel_name": (c_char_p, [_I, _I64, c_int32, c_int32, c_int32, c_int32]),
    "cai_gdn_backward": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, _P, _P, c_int32, _P, c_int32, _P, _P, _F, _F,
                              _P, _P, c_int32, _P, _S, _P]),
    "cai_gdn_backward_deferred": (_I, [_I, _P, c_int32, _P, c_int32, _I64, c_int32, _P, _P, c_int32, _P, c_int32, _P,
                                       _P, _F, _F, _P, _P, c_int32, _P, _S, _P, POINTER(ReduceJob)]),
    "cai_uniform_noise": (_I, [_P, _I64, _P, _P]),
    "cai_quantize": (_I, [_I, _I64, c_int32, _P, _I, c_int32, _P, c_int32, c_int32, _N, _P, _I, c_int32, _P]),
    "cai_gc_fwd": (_I, [_I, _I64, c_int32, _P, _I, c_int32, _P, c_int32, _P, c_int32, _I, _N, _F, _F,
                        _P, _I, c_int32, _P, c_int32, _P]),
    "cai_gc_bwd": (_I, [_I, _I64, c_int32, _P, _I, c_int32, _P, c_int32, _P, c_int32, _I, _N, _F, _F,
                        _P, c_int32, _P, _I, c_int32, _P, c_int32, _P, c_int32, _P, c_int32, _P]),
    "cai_eb_fwd": (_I, [_I, _I64, c_int32, POINTER(EbParams), _P, _I, c_int32, _N, _F, _P, _I, c_int32,
                        _P, c_int32, _P]),
    "cai_eb_scratch_bytes": (_S, [_I64, c_int32]),
    "cai_eb_bwd": (_I, [_I, _I64, c_int32, POINTER(EbParams), _P, _I, c_int32, _N, _F, _P, c_int32, _P,
                        _I, c_int32, _P, c_int32, POINTER(EbGrads), _P, _S, _P, _P]),
    "cai_eb_aux_loss": (_I, [c_int32, POINTER(EbParams), _P, _P, _P, _P, c_int32, _P, _S, _P, _P]),
    "cai_rd_loss_workspace_bytes": (_S, []),
    "cai_rd_loss_fwd": (_I, [POINTER(RdInputs), _F, _F, _P, _P, _S, _P]),
    "cai_rd_loss_bwd": (_I, [POINTER(RdInputs), _F, _F, _P, _P, _P, _P, POINTER(RdGrads), _P]),
    "cai_sum_log": (_I, [_P, _I64, c_int32, c_int32, _P, _P, _S, _P]),
    "cai_sum_sqdiff": (_I, [_P, _P, _I64, _P, _P, _S, _P]),
    "cai_reduce_workspace_bytes": (_S, [_I64]),
    "cai_log_bwd": (_I, [_P, _I64, c_int32, c_int32, _P, _F, _P, _P]),
    "cai_sqdiff_bwd": (_I, [_P, _P, _I64, _P, _F, _P, _P]),
    "cai_sqnorm": (_I, [_P, _I64, _P, _P, _S, _P]),
    "cai_adam": (_I, [_P, _P, _P, _P, _I64, _F, _F, _F, _F, _P, _P, _F, _P]),
    "cai_adam_step_workspace_bytes": (c_size_t, [_I64]),
    "cai_adam_step": (_I, [_P, _P, _P, _P, _I64, _F, _F, _F, _F, _P, _P, _F, c_int32, _P, c_size_t, _P]),
    "cai_act_bwd": (_I, [_I, _F, _P, c_int32, _P, c_int32, _P, c_int32, _I64, c_int32, _I, _P]),
    "cai_cast": (_I, [_P, _I, _P, _I, _I64, _P]),
}


class _Lib:
    def __init__(self):
        self._lib = None

    def load(self):
        if self._lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libcai.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (there is no CPU fallback)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                # an older library missing a newer entry point still serves the
                # others (A/B benches); calling the missing one raises
                fn = getattr(lib, name, None)
                if fn is not None:
                    fn.restype, fn.argtypes = res, args
            self._lib = lib
        return self._lib

    def _bound(self, name):
        return getattr(self.load(), name)

    def __getattr__(self, name):
        fn = self._bound(name)

        if fn.restype is c_int and name not in ("cai_version", "cai_abi_count", "cai_edge_supported",
                                                "cai_conv_split_factor"):
            def call(*args):
                rc = fn(*args)
                if rc != CAI_OK:
                    msg = self._bound("cai_last_error")().decode(errors="replace")
                    if rc in (CAI_EINVAL, CAI_EWORKSPACE):
                        raise ValueError(f"{name}: {msg}")
                    raise RuntimeError(f"{name}: {msg}")
                return rc
            return call
        return fn


lib = _Lib()


def available() -> bool:
    try:
        lib.load()
        return True
    except (OSError, RuntimeError):
        return False
