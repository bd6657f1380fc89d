"""ctypes binding of librecsys_amd.so (C ABI declared in include/recsys_amd.h).

The product path has no fallback: if the shared library is missing or was built for a
different GPU, every op raises. Nothing here imports the CPU oracle.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSX_LIB_PATH") or os.path.join(_HERE, "librecsys_amd.so")  # override: A/B builds

_lock = threading.Lock()
_lib = None
_checked_devices: set = set()

c_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i = ctypes.c_int
c_f = ctypes.c_float
c_u64 = ctypes.c_uint64

ABI_VERSION = 5  # rsx_abi_version() of the library these signatures describe

# name -> (restype, argtypes)
_SIGS = {
    "rsx_last_error": (ctypes.c_char_p, []),
    "rsx_abi_version": (c_i, []),
    "rsx_target_arch": (ctypes.c_char_p, []),
    "rsx_build_hash": (ctypes.c_char_p, []),
    "rsx_seq_embed_fwd": (c_i, [c_p, c_p, c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_i64, c_i64, c_i64, c_f, c_u64,
                                c_p, c_p, c_p, c_p]),
    "rsx_seq_embed_bwd_workspace_floats": (c_i64, [c_i64, c_i64, c_i64]),
    "rsx_seq_embed_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_i64, c_i64,
                                c_i64, c_f, c_u64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "rsx_mha_fwd": (c_i, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i, c_f, c_u64, c_p, c_p, c_p]),
    "rsx_mha_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i, c_f, c_u64, c_p, c_p]),
    "rsx_mha_fwd_x3": (c_i, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i, c_f, c_u64, c_p, c_p, c_p]),
    "rsx_mha_qkv_fwd_x3": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i, c_f, c_u64, c_p, c_p, c_p, c_p]),
    "rsx_mha_bwd_x3": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i, c_f, c_u64, c_p, c_p]),
    "rsx_nce_workspace_floats": (c_i64, [c_i64, c_i64, c_i, c_i]),
    "rsx_nce_fwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_i, c_i, c_p,
                          c_p, c_p]),
    "rsx_nce_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_i, c_i, c_i,
                          c_p, c_p, c_p, c_p, c_i, c_p]),
    "rsx_nce_x3_workspace_floats": (c_i64, [c_i64, c_i64]),
    "rsx_nce_fwd_x3": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_i, c_p, c_p,
                             c_p]),
    "rsx_nce_bwd_x3": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_i, c_p, c_p,
                             c_p, c_p, c_i, c_p]),
    "rsx_nce_emphasis_fwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_f,
                                   c_i, c_i, c_p, c_p, c_p]),
    "rsx_nce_emphasis_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_f,
                                   c_i, c_i, c_p, c_p, c_p, c_p, c_p]),
    "rsx_nce_emphasis_bwd_csr": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f,
                                       c_f, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "rsx_nce_grouped_workspace_floats": (c_i64, [c_i64, c_i64, c_i, c_i, c_i]),
    "rsx_nce_grouped_fwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f, c_i, c_i,
                                  c_p, c_p, c_p]),
    "rsx_kernel_events": (c_i, [c_i]),
    "rsx_kernel_events_read": (c_i, [c_p, c_i]),
    "rsx_gather_events": (c_i, [c_i]),
    "rsx_gather_events_read": (c_i, [c_p, c_p, c_i]),
    "rsx_nce_grouped_fwd_grad": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f, c_i,
                                       c_i, c_p, c_p, c_p, c_p]),
    "rsx_nce_grouped_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                  c_i64, c_i64, c_f, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_i, c_p]),
    "rsx_deepfm_embed": (c_i, [c_p, c_i64, c_i, c_i, c_p, c_p, c_f, c_p, c_p, c_p]),
    "rsx_deepfm_fused_workspace_bytes": (c_i64, [c_i]),
    "rsx_deepfm_fused": (c_i, [c_p, c_i64, c_i, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "rsx_deepfm_fused_prep": (c_i, [c_i, c_p, c_p, c_p, c_p]),
    "rsx_deepfm_fused_run": (c_i, [c_p, c_i64, c_i, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "rsx_deepfm_pack": (c_i, [c_p, c_p, c_i64, c_p, c_p]),
    "rsx_reranker_seq_lens": (c_i, [c_p, c_p, c_i64, c_i, c_p, c_p]),
    "rsx_reranker_batch": (c_i, [c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i64, c_p, c_p, c_p,
                                 c_p, c_p, c_p]),
    "rsx_deepfm_fused_uses_packed": (c_i, [c_i]),
    "rsx_linear_fwd": (c_i, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i, c_p, c_p]),
    "rsx_linear_dot_fwd": (c_i, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i, c_p, c_p, c_p, c_p, c_p]),
    "rsx_static_embed_fwd": (c_i, [c_p, c_p, c_p, c_p, c_i, c_p, c_i64, c_p, c_i64, c_p]),
    "rsx_static_embed_bwd_workspace_floats": (c_i64, [c_i64, c_i, c_p, c_p]),
    "rsx_static_embed_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_i, c_p,
                                   c_i64, c_p]),
    "rsx_dropout_bwd": (c_i, [c_p, c_i64, c_i64, c_f, c_u64, c_p, c_p]),
    "rsx_ln_fwd": (c_i, [c_p, c_p, c_f, c_u64, c_p, c_p, c_f, c_i, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p]),
    "rsx_ln_bwd_workspace_floats": (c_i64, [c_i64, c_i64]),
    "rsx_ln_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_p, c_f, c_u64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p,
                         c_i64, c_p]),
    "rsx_linear_wgrad_workspace_floats": (c_i64, [c_i64, c_i64, c_i64]),
    "rsx_linear_wgrad": (c_i, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i, c_p, c_i64, c_p]),
    "rsx_linear_wgrad_x3": (c_i, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i, c_p, c_i64, c_p]),
    "rsx_gemm_x3": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i, c_p, c_i64, c_f, c_u64, c_p, c_i64, c_p]),
    "rsx_gemm_x3_split_floats": (c_i64, [c_i64, c_i, c_i]),
    "rsx_gemm_x3_ws": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i, c_p, c_i64, c_f, c_u64, c_p, c_i64, c_p,
                             c_i64, c_p]),
    "rsx_gemm_x3_tn": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i, c_p, c_i64, c_f, c_u64, c_p, c_i64,
                             c_p]),
    "rsx_loss_combine": (c_i, [c_p, c_p, c_p, c_p, c_f, c_f, c_f, c_f, c_p, c_p, c_p]),
    "rsx_loss_combine_bwd": (c_i, [c_p, c_p, c_f, c_f, c_f, c_f, c_p, c_p]),
    "rsx_static_profile_arena_bytes": (c_i64, [c_i64]),
    "rsx_static_profile_bwd_workspace_bytes": (c_i64, [c_i64]),
    "rsx_static_profile_fwd": (c_i, [c_p, c_p, c_f, c_f, c_u64, c_p, c_i64, c_p, c_p]),
    "rsx_static_profile_bwd": (c_i, [c_p, c_p, c_f, c_u64, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "rsx_clip_adamw_workspace_bytes": (c_i64, [c_i, c_p, c_p]),
    "rsx_clip_adamw": (c_i, [c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_i64,
                             c_p, c_p]),
    "rsx_tower_n_ptrs": (c_i64, [c_i]),
    "rsx_tower_arena_bytes": (c_i64, [c_i64, c_i64, c_i]),
    "rsx_tower_bwd_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64, c_i, c_i64]),
    "rsx_tower_fwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p]),
    "rsx_tower_bwd": (c_i, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "rsx_gemm_x3_rowadd": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_i, c_p, c_i64, c_p, c_p, c_i64, c_p]),
    "rsx_gemm_x3_addln": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_i, c_p, c_i64, c_f, c_u64, c_p, c_p, c_f,
                                c_p, c_i64, c_p, c_i64, c_p, c_p, c_p]),
    "rsx_topk_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "rsx_retrieve_topk": (c_i, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p]),
    "rsx_topk_path": (c_i, [c_i64, c_i64, c_i64]),
    "rsx_ids_check": (c_i, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "rsx_step_index_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "rsx_step_index_count": (c_i, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p]),
    "rsx_step_index_totals": (c_i, [c_p, c_i, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p]),
    "rsx_step_index_fill": (c_i, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_i64, c_p, c_p]),
    "rsx_topk_corpus_bytes": (c_i64, [c_i64]),
    "rsx_topk_prepare_corpus": (c_i, [c_p, c_i64, c_i64, c_p, c_p]),
    "rsx_topk_workspace_bytes_corpus": (c_i64, [c_i64, c_i64, c_i64]),
    "rsx_retrieve_topk_corpus": (c_i, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p]),
    "rsx_gather_rows": (c_i, [c_p, c_i64, c_p, c_i64, c_i64, c_i, c_f, c_p, c_p, c_p]),
    "rsx_embed3_ln": (c_i, [c_p, c_i64, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_i64, c_i64, c_p, c_p]),
    "rsx_crossnet": (c_i, [c_p, c_i64, c_i64, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p]),
    "rsx_segment_sum_rows": (c_i, [c_p, c_i64, c_p, c_p, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i, c_p]),
    "rsx_scatter_rows": (c_i, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i, c_f, c_i, c_i64, c_p, c_i64, c_p]),
    "rsx_hnm_mine": (c_i, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f, c_f, c_p, ctypes.c_size_t, c_p, c_p, c_p, c_p]),
    "rsx_hnm_workspace_bytes": (c_i64, [c_i64]),
    "rsx_hnm_max_rows": (c_i64, []),
}

EXPORTED_SYMBOLS = tuple(_SIGS.keys())


def load(path: str = LIB_PATH):
    """Load and type the library (idempotent). Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"recsys_amd: native library not found at {path}; run __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rsx_abi_version() != ABI_VERSION:
            raise RuntimeError(f"recsys_amd: {path} has ABI {lib.rsx_abi_version()}, this binding expects "
                               f"{ABI_VERSION}; rebuild with __graft_entry__.build()")
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load()


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the library's sources in this tree, in csrc/Makefile's order
    (the .hip files sorted by name, rsx_common.h, include/recsys_amd.h): equal to
    rsx_build_hash() of a library built from them."""
    import glob
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")), key=lambda f: os.path.basename(f).encode())
    files += [os.path.join(csrc, "rsx_common.h"),
              os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "recsys_amd.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info() -> dict:
    """The loaded library's source stamp against this tree's sources (fresh = built from them)."""
    built = lib().rsx_build_hash().decode()
    src = source_hash()
    return {"lib_hash": built, "src_hash": src, "fresh": built == src}


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().rsx_last_error().decode(errors="replace")
        raise RuntimeError(f"recsys_amd {what} failed (code {rc}): {msg}")


def ensure_device(t: torch.Tensor) -> None:
    """The kernels are gfx950 code objects: refuse anything else loudly."""
    if t.device.type != "cuda":
        raise RuntimeError(f"recsys_amd ops need a ROCm GPU tensor, got device {t.device}")
    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if idx in _checked_devices:
        return
    arch = torch.cuda.get_device_properties(idx).gcnArchName.split(":")[0]
    want = lib().rsx_target_arch().decode()
    if arch != want:
        raise RuntimeError(f"recsys_amd was built for {want} but device {idx} is {arch}")
    _checked_devices.add(idx)


def stream() -> int:
    """The current HIP stream of the current device, as a raw pointer. The raw query skips the
    torch.cuda.Stream object that current_stream() builds per call (~33 native calls per train
    step: 0.3 ms of host time per step in the unloaded-step profile)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def ptr_array(tensors, ctype=ctypes.c_void_p):
    arr = (ctype * max(1, len(tensors)))()
    for k, t in enumerate(tensors):
        arr[k] = None if t is None else t.data_ptr()
    return arr


def i64_array(vals):
    arr = (ctypes.c_int64 * max(1, len(vals)))()
    for k, v in enumerate(vals):
        arr[k] = int(v)
    return arr
