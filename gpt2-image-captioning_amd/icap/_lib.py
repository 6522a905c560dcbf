"""ctypes binding of libicap_hip.so (C-ABI declared in include/icap.h).

The library is the product path: there is no CPU or PyTorch fallback. If the
shared object is missing, or its gfx950 code object cannot be loaded on the
current device, every op raises.
"""

from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must be imported first: the .so binds to torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ICAP_LIB: another build of the same ABI (diagnostic builds for tools/: the -DICAP_STAMPS library)
LIB_PATH = os.environ.get("ICAP_LIB") or os.path.join(_HERE, "libicap_hip.so")

F32, BF16, FP8_MX = 0, 1, 2
ACT_NONE, ACT_GELU_NEW, ACT_RELU, ACT_QUICK_GELU, ACT_TANH, ACT_GELU_ERF = 0, 1, 2, 3, 4, 5

vp = C.c_void_p
i32, i64, u64, f32, sz = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
pi32 = C.POINTER(C.c_int32)
pi64 = C.POINTER(C.c_int64)


class GemmArgs(C.Structure):
    _fields_ = [
        ("M", i64), ("N", i64), ("K", i64),
        ("in_dtype", i32), ("c_dtype", i32),
        ("A", vp), ("lda", i64),
        ("B", vp), ("ldb", i64),
        ("C", vp), ("ldc", i64),
        ("alpha", f32), ("beta", f32),
        ("bias", vp),
        ("act", i32),
        ("aux", vp), ("ldaux", i64),
        ("dact", i32),
        ("dact_src", vp), ("ld_dact", i64),
        ("resid", vp), ("ldr", i64),
        ("drop_p", f32), ("seed", u64), ("offset", u64),
        ("seed_ptr", vp),
        ("workspace", vp), ("workspace_bytes", i64), ("split_k", i32),
        ("m_dev", vp),
        ("trans_ab", i32),
        ("ln_gamma", vp), ("ln_beta", vp), ("ln_eps", f32),
        ("path", i32),
        ("a_scale", vp), ("b_scale", vp),
        ("m_hint", i64),
        ("tickets", vp), ("tickets_len", i64),
        ("ln_wsum", vp),
        ("ln_stats_out", vp), ("ln_stats_in", vp), ("ln_mean_out", vp), ("ln_rstd_out", vp),
        ("diag_stamps", vp),
    ]


class LnParamItem(C.Structure):
    _fields_ = [("workspace", vp), ("rows", i64), ("D", i64), ("dgamma", vp), ("dbeta", vp), ("overwrite", i32)]


class TransposeItem(C.Structure):
    _fields_ = [("src", vp), ("lds", i64), ("dst", vp), ("ldd", i64), ("rows", i64), ("cols", i64)]


class ColsumItem(C.Structure):
    _fields_ = [("src", vp), ("ld", i64), ("N", i64), ("out", vp)]


class AttnArgs(C.Structure):
    _fields_ = [
        ("dtype", i32),
        ("B", i32), ("S", i32), ("H", i32), ("hd", i32),
        ("row_stride_b", i64), ("row_stride_s", i64),
        ("qkv", vp), ("ld_qkv", i64),
        ("out", vp), ("ld_out", i64),
        ("lse", vp),
        ("key_mask", vp),
        ("causal", i32),
        ("scale", f32),
        ("drop_p", f32), ("seed", u64), ("offset", u64),
        ("seed_ptr", vp),
        ("dout", vp), ("ld_dout", i64),
        ("dqkv", vp), ("ld_dqkv", i64),
        ("seq_off", vp), ("seq_len", vp),
        ("short_only", i32),
    ]


class AdamWArgs(C.Structure):
    _fields_ = [
        ("n", i64),
        ("params", vp), ("grads", vp), ("exp_avg", vp), ("exp_avg_sq", vp),
        ("bf16_out", vp),
        ("state", vp),
        ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32),
        ("max_norm", f32),
        ("num_warmup_steps", i64), ("num_training_steps", i64),
    ]


class BeamArgs(C.Structure):
    _fields_ = [
        ("B", i32), ("W", i32), ("V", i32), ("max_len", i32),
        ("eos", i32), ("length_penalty", f32),
        ("K", i32),
        ("T", i32),
        ("top_val", vp), ("top_idx", vp), ("top_m", vp), ("top_ls", vp),
        ("ws", vp),
        ("dtype", i32), ("D", i32), ("n_positions", i32),
        ("wte", vp), ("wpe", vp), ("x", vp),
    ]


# name -> (restype, argtypes); must mirror include/icap.h exactly
SIGNATURES = {
    "icap_last_error": (C.c_char_p, []),
    "icap_version": (C.c_int, []),
    "icap_device_arch_ok": (C.c_int, []),
    "icap_gemm": (C.c_int, [C.POINTER(GemmArgs), vp]),
    "icap_gemm_group": (C.c_int, [C.POINTER(GemmArgs), C.c_int32, vp]),
    "icap_gemm_kernel_name": (C.c_char_p, [C.POINTER(GemmArgs)]),
    "icap_gemm_plan_info": (C.c_int, [C.POINTER(GemmArgs), vp, vp]),
    "icap_mx_scale_bytes": (sz, [i64, i64]),
    "icap_quantize_mx": (C.c_int, [i32, i64, i64, vp, i64, vp, i64, vp, vp, vp]),
    "icap_layernorm_fwd": (C.c_int, [i32, i64, i64, vp, i64, vp, vp, f32, vp, i64, vp, vp, vp, vp, vp]),
    "icap_layernorm_bwd_workspace_bytes": (sz, [i64, i64]),
    "icap_layernorm_bwd": (C.c_int, [i32, i64, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, i64, vp,
                                     f32, u64, u64, vp, vp, vp, vp, vp, vp, i32, vp]),
    "icap_ln_param_reduce_batch": (C.c_int, [i32, C.POINTER(LnParamItem), vp]),
    "icap_attention_fwd": (C.c_int, [C.POINTER(AttnArgs), vp]),
    "icap_attention_bwd": (C.c_int, [C.POINTER(AttnArgs), vp]),
    "icap_attention_decode": (C.c_int, [i32, i32, i32, i32, i32, vp, i64, vp, i64, f32, vp]),
    "icap_attention_decode_anc": (C.c_int, [i32, i32, i32, i32, i32, vp, i64, vp, vp, i64, f32, vp]),
    "icap_beam_workspace_bytes": (C.c_size_t, [i32, i32, i32, i32]),
    "icap_beam_layout": (C.c_int, [i32, i32, i32, i32, vp]),
    "icap_beam_init": (C.c_int, [C.POINTER(BeamArgs), i32, vp]),
    "icap_beam_rowtop": (C.c_int, [i32, i64, i64, vp, i64, i32, vp, vp, vp, vp, vp]),
    "icap_beam_update": (C.c_int, [C.POINTER(BeamArgs), i32, i32, vp]),
    "icap_beam_finalize": (C.c_int, [C.POINTER(BeamArgs), vp, vp, vp]),
    "icap_gpt2_embed": (C.c_int, [i32, i32, i32, i32, i32, vp, i64, vp, vp, vp, vp, f32, u64, u64, vp, vp, vp, vp]),
    "icap_embedding_scatter_add": (C.c_int, [i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    "icap_caption_prep": (C.c_int, [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    "icap_caption_pack": (C.c_int, [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "icap_rows_unpack": (C.c_int, [i32, i32, i32, i32, vp, vp, vp, vp, i64, vp]),
    "icap_cross_entropy_workspace_bytes": (sz, [i64]),
    "icap_cross_entropy": (C.c_int, [i32, i64, i64, vp, i64, vp, vp, vp, vp, f32, vp, vp, vp]),
    "icap_adamw_workspace_bytes": (sz, [i64]),
    "icap_adamw_step": (C.c_int, [C.POINTER(AdamWArgs), vp, vp]),
    "icap_sqnorm": (C.c_int, [i64, vp, vp, vp, vp]),
    "icap_transpose": (C.c_int, [i32, i64, i64, vp, i64, vp, i64, i64, vp]),
    "icap_transpose_batch": (C.c_int, [i32, vp, vp]),
    "icap_colsum_workspace_bytes": (sz, [i64, i64]),
    "icap_colsum": (C.c_int, [i32, i64, i64, vp, i64, vp, i32, vp, vp]),
    "icap_colsum_batch": (C.c_int, [i32, i64, i32, vp, i32, vp, vp]),
    "icap_dropout_apply": (C.c_int, [i32, i64, i64, vp, i64, vp, i64, f32, u64, u64, vp, vp]),
    "icap_counter_increment": (C.c_int, [vp, vp]),
    "icap_convert": (C.c_int, [i32, i32, i64, i64, vp, i64, vp, i64, vp]),
    "icap_broadcast_rows": (C.c_int, [i32, i32, i64, i64, vp, vp, i64, vp]),
    "icap_im2col_patches": (C.c_int, [i32, i32, i32, i32, i32, vp, vp, vp]),
    "icap_vit_embed": (C.c_int, [i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    "icap_prefix_embed": (C.c_int, [i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    "icap_patch_embed": (C.c_int, [i32, i32, i32, i32, i32, i32, vp, vp, i64, i32, vp, vp, vp, vp, i64, vp]),
    "icap_rope_patches": (C.c_int, [i32, i32, i32, i32, i32, i32, vp, i64, vp, vp, vp]),
    "icap_l2norm_rows": (C.c_int, [i32, i64, i64, vp, i64, vp, i64, vp]),
    "icap_topp_sample": (C.c_int, [i32, i32, i64, vp, i64, f32, f32, vp, u64, vp, i32, i64, vp, vp]),
    "icap_greedy_next": (C.c_int, [i32, i32, i64, vp, i64, i64, vp, vp, vp, i64, i32, vp, vp, i32, i32, vp, vp]),
    "icap_add_position": (C.c_int, [i32, i32, i32, i32, vp, i64, i64, vp, i32, vp, vp]),
    "icap_clip_preprocess": (C.c_int, [i32, vp, vp, i32, i32, vp, vp, vp, vp, vp]),
}

_lib = None


class IcapError(RuntimeError):
    pass


def load(path: str = LIB_PATH, strict: bool = True) -> C.CDLL:
    """Load (once) and bind the library; raises if it is missing. strict=False (A/B measurement tools loading an
    older build) skips entry points the build does not export."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise IcapError(
            f"libicap_hip.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no fallback path)"
        )
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().icap_last_error()
    return msg.decode() if msg else ""


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise IcapError(f"{name} failed ({rc}): {last_error()}")


_device_checked = set()


def require_device(dev: torch.device) -> None:
    """Fail loudly unless `dev` is a GPU on which the gfx950 code object loads."""
    if dev.type != "cuda":
        raise IcapError(f"icap kernels run on the GPU only (got device {dev}); there is no CPU fallback")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _device_checked:
        return
    lib = load()
    with torch.cuda.device(idx):
        if not lib.icap_device_arch_ok():
            raise IcapError(f"libicap_hip.so code object not loadable on device {idx}: {last_error()}")
    _device_checked.add(idx)
