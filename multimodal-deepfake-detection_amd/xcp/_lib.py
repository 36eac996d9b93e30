"""ctypes binding of the C ABI in ``include/xcp.h`` (``libxcp.so``).

This is the reference-side binding a maintainer would add: the
reference reaches these ops only implicitly through ``torch.nn``; here every
entry point is bound by name with explicit argument types.  Loading fails
loudly when the library is missing -- there is no fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = DEFAULT_LIB_PATH = os.path.join(_HERE, "libxcp.so")
# XCP_LIB_PATH: load another build of the same ABI instead (A/B of a kernel change in the step;
# tools/build_variant.py links one).  A development switch: honoured only for a file inside this
# repository's tree, announced on stderr at load with every entry point the build lacks.
_REPO = os.path.dirname(os.path.dirname(_HERE))
_OVERRIDE = os.environ.get("XCP_LIB_PATH")
if _OVERRIDE:
    _real = os.path.realpath(_OVERRIDE)
    if os.path.commonpath([_real, os.path.realpath(_REPO)]) != os.path.realpath(_REPO):
        raise ImportError(f"XCP_LIB_PATH={_OVERRIDE} is outside the repository ({_REPO}); "
                          "only in-tree A/B builds may replace libxcp.so")
    LIB_PATH = _real
MISSING = []   # entry points an XCP_LIB_PATH build lacks (calling one raises XcpError)

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
D = ctypes.c_double

# name -> argument types (return type is always int status)
SIGNATURES = {
    "xcp_gemm_nt": [I, P, L, P, L, P, L, I, I, I, P, I, I, I, I, I, I, I, I, P],
    "xcp_gemm_nt_stat_rows": [I],
    "xcp_gemm_tn_rows_per_split": [I, I, I, I, I, I],
    "xcp_gemm_tn": [I, P, L, P, L, P, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "xcp_unit_bwd_rows_per_split": [I, I, I, I],
    "xcp_unit_bwd": [I, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "xcp_dw_fwd": [I, I, P, P, P, P, P, I, I, I, I, P],
    "xcp_sep_fwd_parts": [I, I, I, I, I, I],
    "xcp_sep_fwd": [I, I, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "xcp_dw_bwd_chunks": [I, I, I, I],
    "xcp_dw_bwd": [I, I, P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, I, I, I, I, P],
    "xcp_dw_bwd_resbn": [I, I, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "xcp_colreduce_f32": [P, I, L, L, P, I, I, P],
    "xcp_colreduce_groups": [I, L],
    "xcp_colreduce_multi": [P, I, P],
    "xcp_chanred_parts": [L, I],
    "xcp_row_stats": [I, P, L, I, P, P],
    "xcp_bn_bwd_reduce": [I, P, P, P, P, P, P, L, I, P, P],
    "xcp_bn_finalize_part": [P, I, I, I, D, P, P, P, P, F, F, P, P, P, P, P],
    "xcp_bn_bwd_finalize_part": [P, I, I, I, D, P, P, P, P, P, P, P, P, I, P],
    "xcp_bn_finalize": [P, I, I, I, D, P, P, P, P, F, F, I, P, P, P, P, P],
    "xcp_bn_act": [I, P, P, P, P, I, L, I, P],
    "xcp_bn_act_strided": [I, P, P, P, P, I, I, I, I, I, I, I, I, P],
    "xcp_bn_bwd_apply": [I, P, P, P, P, P, P, P, P, L, I, P],
    "xcp_relu_bwd": [I, P, P, L, I, P],
    "xcp_tail_fwd": [I, P, P, P, I, P, P, P, P, P, I, I, I, I, P],
    "xcp_maxpool_bwd": [I, P, P, P, I, I, I, I, P],
    "xcp_maxpool_bwd_bnred_parts": [I, I, I, I],
    "xcp_maxpool_bwd_bnred": [I, P, P, P, P, P, P, I, I, I, I, P, P],
    "xcp_avgpool_fwd": [I, P, P, P, P, I, I, I, P],
    "xcp_avgpool_bwd": [I, P, P, P, P, P, I, I, I, P],
    "xcp_conv1_fwd": [I, P, P, P, I, I, I, P],
    "xcp_conv1_fwd_parts": [I, I, I],
    "xcp_conv1_fwd_stats": [I, P, P, P, P, I, I, I, P],
    "xcp_conv1_wgrad_parts": [I, I, I],
    "xcp_conv1_wgrad": [I, P, P, P, I, I, I, P],
    "xcp_conv1_wgrad_fused": [I, I, I],
    "xcp_conv1_wgrad_bn": [I, P, P, P, P, P, P, P, P, P, I, I, I, P],
    "xcp_permute3": [I, P, P, I, I, I, I, I, I, P],
    "xcp_permute3_blocks": [I, I, I, I, I, I, L, L],
    "xcp_permute3_batch": [P, I, I, P],
    "xcp_frames_u8_to_f32": [P, P, P, I, I, I, I, P],
    "xcp_resize_bilinear": [P, P, I, I, I, I, I, P],
    "xcp_frames_prep": [P, P, P, I, I, I, I, I, I, I, I, P],
    "xcp_opt_sumsq": [P, I, P, F, P, P],
    "xcp_opt_adam": [P, I, P, F, F, F, F, F, F, F, P],
    "xcp_opt_adam_dev": [P, I, P, F, D, D, F, F, P, P],
    "xcp_conv3x3_parts": [I, I, I, I],
    "xcp_conv3x3": [I, P, P, P, P, I, I, I, P, P, P],
    "xcp_conv3x3_wgrad_parts": [I, I, I],
    "xcp_conv3x3_wgrad": [P, P, P, I, I, I, P, P, P],
    "xcp_arcface_fwd": [P, P, P, P, I, I, I, F, F, P],
    "xcp_arcface_bwd": [P, P, P, P, P, P, I, I, I, F, F, P],
    "xcp_focal_ce": [P, P, P, F, P, P, P, I, I, P],
    "xcp_lstm_needs_whhT": [I, I, I],
    "xcp_lstm_fwd": [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "xcp_lstm_bwd": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "xcp_lstm_sync_error": [],
    "xcp_clock_probe": [P, I, I, P],
    "xcp_stream_copy": [P, P, L, P],
    "xcp_comm_proxy": [P, P, L, I, ctypes.c_longlong, P, P],
    "xcp_stamp": [P, P],
}

# entry points that return a size, not a status
SIZE_QUERIES = {"xcp_permute3_blocks", "xcp_sep_fwd_parts", "xcp_gemm_tn_rows_per_split", "xcp_gemm_nt_stat_rows", "xcp_dw_bwd_chunks", "xcp_chanred_parts",
                "xcp_colreduce_groups", "xcp_unit_bwd_rows_per_split",
                "xcp_conv1_wgrad_parts", "xcp_conv1_wgrad_fused", "xcp_conv1_fwd_parts", "xcp_lstm_needs_whhT", "xcp_conv3x3_parts", "xcp_conv3x3_wgrad_parts",
                "xcp_maxpool_bwd_bnred_parts", "xcp_lstm_sync_error"}

_lib = None


class XcpError(RuntimeError):
    pass


def load():
    """Load libxcp.so (after torch, so the process shares torch's HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- HIP runtime of torch must be the one resolved
    if not os.path.exists(LIB_PATH):
        raise XcpError(f"HIP library {LIB_PATH} is missing; run `python -m xcp.build` (hipcc, gfx950). "
                       "There is no CPU fallback for the product path.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        if LIB_PATH != DEFAULT_LIB_PATH and not hasattr(lib, name):
            MISSING.append(name)   # an A/B build of an older tree (XCP_LIB_PATH) may predate an entry point
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    if LIB_PATH != DEFAULT_LIB_PATH:
        import sys
        print(f"xcp: XCP_LIB_PATH override {LIB_PATH}; entry points it lacks: {MISSING or 'none'}",
              file=sys.stderr)
    _lib = lib
    return lib


def call(name, *args):
    """Call an entry point; raise XcpError on a non-zero status."""
    lib = load()
    if MISSING and name in MISSING:
        raise XcpError(f"{name} is not in the XCP_LIB_PATH build {LIB_PATH}")
    fn = getattr(lib, name)
    rc = fn(*args)
    if name in SIZE_QUERIES:
        return rc
    if rc != 0:
        raise XcpError(f"{name} failed with status {rc}")
    return rc
