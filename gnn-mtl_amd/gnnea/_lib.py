"""ctypes binding of libgnnea.so (the C-ABI declared in include/gnnea.h).

The library is loaded after ``import torch`` so that it binds to the HIP runtime torch already
loaded (same soname, ``libamdhip64.so.7``): device pointers and streams are shared.  There is no
fallback: if the library is missing every product op raises.
"""
import contextlib
import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library is dlopen'ed)

_HERE = os.path.dirname(os.path.abspath(__file__))
# GNNEA_LIB_FILE: another build of the library next to this one (A/B timing of variant builds
# only; a file name, not a path)
LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("GNNEA_LIB_FILE", "libgnnea.so")))

GNNEA_ACT_IDENTITY = 0
GNNEA_ACT_RELU = 1
GNNEA_ACT_ELU = 2
GNNEA_ACT_LEAKY_RELU = 3
GNNEA_ACT_SIGMOID = 4
GNNEA_ACT_TANH = 5
GNNEA_UB_NT = 1  # gnnea_ub_copy flags (include/gnnea.h)
GNNEA_UB_DEEP = 2
GNNEA_UB_READ_ONLY = 4
GNNEA_UB_GAT_WIN12 = 1  # gnnea_ub_gather modes
GNNEA_UB_GAT_V16 = 2

GNNEA_F32 = 0
GNNEA_F64 = 1
GNNEA_BF16 = 2

GNNEA_SK_KNOPP = 0
GNNEA_SK_STAB = 1
GNNEA_SK_GEN = 2
GNNEA_SK_RELAX = 3
GNNEA_SK_STATUS_BYTES = 256
GNNEA_SK_PATH_SWEEP, GNNEA_SK_PATH_ONCHIP, GNNEA_SK_PATH_LOG = 0, 1, 2
GNNEA_SK_ST_TIMEOUT = 16  # status word: an inter-workgroup wait of k_sk_res timed out
GNNEA_SK_NO_ONCHIP = 1  # gnnea_sinkhorn.flags: never the on-chip persistent path
GNNEA_SK_TWO_PASS = 2  # gnnea_sinkhorn.flags: KNOPP log domain as two passes (not the fused sweep)
GNNEA_SK_DEBUG_SPIN = 4  # gnnea_sinkhorn.flags: zero wait budget on chip (timeout-path tests)
GNNEA_SK_AUTO = 3  # gnnea_sinkhorn.variant: on chip / fused log-domain sweep / scaling form

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_f64 = ctypes.c_double


class SinkhornProblem(ctypes.Structure):
    """Mirror of ``gnnea_sinkhorn`` (include/gnnea.h)."""

    _fields_ = [
        ("mode", ctypes.c_int),
        ("c_dtype", ctypes.c_int),
        ("I", ctypes.c_int),
        ("J", ctypes.c_int),
        ("ldc", _i64),
        ("C", _p),
        ("a", _p),
        ("b", _p),
        ("eps", _f64),
        ("p", _f64),
        ("tol", _f64),
        ("max_iter", ctypes.c_int),
        ("iters_run", ctypes.c_int),
        ("variant", ctypes.c_int),
        ("flags", ctypes.c_int),
        ("ws", _p),
    ]


# name -> (restype, argtypes): every symbol include/gnnea.h declares
SIGNATURES = {
    "gnnea_abi_version": (ctypes.c_int, []),
    "gnnea_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gnnea_coo_to_csr_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_coo_to_csr": (ctypes.c_int, [_p, _p, ctypes.c_int, _p, _i64, _i64, _i64, _p, _p, _p,
                                        _p, _p, _p, _i64, _p]),
    "gnnea_csr_expand_rows": (ctypes.c_int, [_p, _i32, _i64, _p, _p]),
    "gnnea_perm_invert": (ctypes.c_int, [_p, _i64, _p, _p]),
    "gnnea_spmm_csr_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64,
                                          ctypes.c_int, _p]),
    "gnnea_spmm_csr_beta_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _f32, _p, _i64,
                                               ctypes.c_int, _p]),
    "gnnea_spmm_sliced_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64,
                                             ctypes.c_int, _p]),
    "gnnea_spmm_highway_sliced_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64,
                                                     _i32, _p, _p, _i64, _p, _i64, _p, _p, _i64,
                                                     ctypes.c_int, _p]),
    "gnnea_highway_bwd_sliced_f32": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i32, _p, _i64,
                                                    _p, _i64, _p, _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_sliced_zg_f32": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _p, _p, _i64, _i64,
                                                       _i32, _p, _i64, _p, _i64, _p, _i64,
                                                       ctypes.c_int, _p]),
    "gnnea_spmm_highway_sliced_m_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p,
                                                       _i64, _i32, _p, _p, _i64, _p, _i64, _p,
                                                       _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_sliced_zgm_f32": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _p, _p, _i64,
                                                        _i64, _i32, _p, _i64, _p, _i64, _p, _i64,
                                                        _p, _i64, ctypes.c_int, _p]),
    "gnnea_spmm_sliced_bf16": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64,
                                              ctypes.c_int, ctypes.c_int, _p]),
    "gnnea_slice_pack_bf16": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _i64, _p]),
    "gnnea_spmm_sliced64_bf16": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64,
                                                ctypes.c_int, ctypes.c_int, _p]),
    "gnnea_act_bwd_sliced_bf16": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i32, ctypes.c_int,
                                                 _p, _i64, _p]),
    "gnnea_slice_pack_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _i64, _p]),
    "gnnea_act_bwd_sliced_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i32, ctypes.c_int, _p,
                                                _i64, _p]),
    "gnnea_spmm_highway_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64, _p, _p,
                                              _i64, _p, _i64, _p, _p, _i64, ctypes.c_int, _p]),
    "gnnea_act_bwd_f32": (ctypes.c_int, [_p, _p, _p, _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_ld_f32": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i32, _p, _i64, _p,
                                                 _i64, _p, _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_f32": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p,
                                             ctypes.c_int, _p]),
    "gnnea_spmm_csr_bf16": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _f32, _p, _i64,
                                           ctypes.c_int, ctypes.c_int, _p]),
    "gnnea_spmm_highway_bf16": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64, _p,
                                               _p, _i64, _p, _i64, _p, _p, _i64, ctypes.c_int,
                                               _p]),
    "gnnea_act_bwd_bf16": (ctypes.c_int, [_p, _p, _p, _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_ld_bf16": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i32, _p, _i64, _p,
                                                  _i64, _p, _i64, ctypes.c_int, _p]),
    "gnnea_highway_bwd_bf16": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p,
                                              ctypes.c_int, _p]),
    "gnnea_gat_scores_f32": (ctypes.c_int, [_p, _i64, _i32, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                            _p]),
    "gnnea_gat_scores_bf16": (ctypes.c_int, [_p, _i64, _i32, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                            _p]),
    "gnnea_gat_fwd_f32": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int, ctypes.c_int, _p, _p,
                                         _f32, _p, ctypes.c_int, _p, _i64, _p, _p, _p]),
    "gnnea_gat_fwd_bf16": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int, ctypes.c_int, _p, _p,
                                         _f32, _p, ctypes.c_int, _p, _i64, _p, _p, _p]),
    "gnnea_gat_bwd_prep_f32": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.c_int, _p, _p, _i64, _p,
                                              _p, _p, ctypes.c_int, _p, _p, _p]),
    "gnnea_gat_bwd_prep_bf16": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.c_int, _p, _p, _i64, _p,
                                              _p, _p, ctypes.c_int, _p, _p, _p]),
    "gnnea_gat_bwd_src_f32": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int, ctypes.c_int, _p, _i64,
                                             _p, _f32, _p, _p, _p, _i64, _p, _p, _i64, _p, _p, _p]),
    "gnnea_gat_bwd_src_bf16": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int, ctypes.c_int, _p, _i64,
                                             _p, _f32, _p, _p, _p, _i64, _p, _p, _i64, _p, _p, _p]),
    "gnnea_gat_bwd_src_rows_bf16": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int, ctypes.c_int,
                                                   _p, _i64, _p, _f32, _p, _p, _p, _i64, _i64, _p,
                                                   _p, _i64, _p, _p, _p]),
    "gnnea_gat_bwd_dst_f32": (ctypes.c_int, [_p, _p, _i32, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                             _i64, _p, _p]),
    "gnnea_gat_bwd_dst_bf16": (ctypes.c_int, [_p, _p, _i32, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                             _i64, _p, _p]),
    "gnnea_gat_da_ws_bytes": (_i64, [_i64, _i32]),
    "gnnea_gat_da_f32": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                        _i64, _p]),
    "gnnea_gat_da_bf16": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                         _i64, _p]),
    "gnnea_gat_da2_f32": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                         _p, _p, _i64, _p]),
    "gnnea_gat_da2_bf16": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                          _p, _p, _i64, _p]),
    "gnnea_colsum_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _i64, _p]),
    "gnnea_act_fwd_f32": (ctypes.c_int, [_p, _p, _i64, ctypes.c_int, _p]),
    "gnnea_act_fwd_bf16": (ctypes.c_int, [_p, _p, _i64, ctypes.c_int, _p]),
    "gnnea_head_mean_f32": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _i64,
                                           ctypes.c_int, _p]),
    "gnnea_head_mean_bf16": (ctypes.c_int, [_p, _i64, _i64, ctypes.c_int, ctypes.c_int, _p, _i64,
                                            ctypes.c_int, _p]),
    "gnnea_act_bwd_colsum_ws_bytes": (_i64, [_i64, _i32]),
    "gnnea_act_bwd_colsum_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i32, ctypes.c_int, _p,
                                                _i64, _p, _p, _i64, _p]),
    "gnnea_act_bwd_colsum_bf16": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i32, ctypes.c_int, _p,
                                                 _i64, _p, _p, _i64, _p]),
    "gnnea_gemm_bf16_dmask_applies": (ctypes.c_int, [_i64, _i64, _i64, _i64, _i64, _i64]),
    "gnnea_gemm_bf16_dmask_ws_bytes": (_i64, [_i64, _i64]),
    "gnnea_gemm_bf16_dmask": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p, _i64,
                                             _p, _i64, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_bf16_mask_ld": (_i64, [_i64]),
    "gnnea_gemm_bf16_relu_mask": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                                 _i64, _p, _p, _i64, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_bf16_dmask_bits": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                                  _i64, _p, _i64, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_f32_mask_applies": (ctypes.c_int, [_i64, _i64, _i64, _i64, _i64]),
    "gnnea_gemm_f32_mask_ld": (_i64, [_i64]),
    "gnnea_gemm_f32_mask_ws_bytes": (_i64, [_i64]),
    "gnnea_gemm_f32_relu_mask": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                                _i64, _p, _p, _i64, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_f32_dmask_bits": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                                 _i64, _p, _i64, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_x3_ta_db_applies": (ctypes.c_int, [_i64, _i64, _i64, _i64, _i64]),
    "gnnea_gemm_x3_ta_db_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_gemm_x3_ta_db_f32": (ctypes.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p,
                                               _p, _i64, _p]),
    "gnnea_gemm_bf16_ta_db_applies": (ctypes.c_int, [_i64, _i64, _i64, _i64, _i64]),
    "gnnea_gemm_bf16_ta_db": (ctypes.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64,
                                             ctypes.c_int, _p, _p, _i64, _p]),
    "gnnea_spmm_sliced_m_f32": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i64, _p, _i64, _p,
                                               _i64, _p]),
    "gnnea_act_bwd_sliced_bits_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i32, _p, _i64,
                                                     _p]),
    "gnnea_gemm_bf16_act": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p, _i64,
                                           _p, _i64, _p, ctypes.c_int, _p, _i64, ctypes.c_int, _p,
                                           _i64, _p]),
    "gnnea_gemm_x3_act_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p,
                                             _i64, _p, _i64, _p, ctypes.c_int, _p, _i64, _p, _i64,
                                             _p]),
    "gnnea_colsum_bf16": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _i64, _p]),
    "gnnea_gemm_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_gemm_bf16_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_gemm_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                       _i64, _p, _f32, _p, _i64, ctypes.c_int, _p, _i64, _p]),
    "gnnea_gemm_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                      _i64, _p, _f32, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_sliced_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p,
                                             _i64, _p, _i64, _p, _f32, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_sliced_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p,
                                              _i64, _p, _i64, _p, _f32, _p, _i64, _p, _i64, _p]),
    "gnnea_gat_fwd_sliced_f32": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int,
                                                ctypes.c_int, _p, _p, _f32, _p, ctypes.c_int, _p,
                                                _i64, _p, _p, _p, _p]),
    "gnnea_gat_bwd_prep_sliced_f32": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.c_int, _p, _p,
                                                     _i64, _p, _p, _p, ctypes.c_int, _p, _i64, _p,
                                                     _p]),
    "gnnea_gat_bwd_src_sliced_f32": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int, ctypes.c_int,
                                                    _p, _i64, _p, _f32, _p, _p, _p, _i64, _p, _p,
                                                    _i64, _p, _i64, _p]),
    "gnnea_gat_bwd_edge_sliced_f32": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int, ctypes.c_int,
                                                     _p, _f32, _p, _p, _p, _i64, _p, _p, _i64, _p,
                                                     _p, _p]),
    "gnnea_gat_bwd_dst_sliced_f32": (ctypes.c_int, [_p, _p, _i32, ctypes.c_int, ctypes.c_int, _p,
                                                    _p, _p, _p, _i64, _p, _p]),
    "gnnea_gat_fwd_sliced_bf16": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int,
                                                 ctypes.c_int, _p, _p, _f32, _p, ctypes.c_int, _p,
                                                 _i64, _p, _p, _p, _p]),
    "gnnea_gat_bwd_prep_sliced_bf16": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.c_int, _p, _p,
                                                      _i64, _p, _p, _p, ctypes.c_int, _p, _i64,
                                                      _p, _p]),
    "gnnea_gat_bwd_src_sliced_bf16": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int,
                                                     ctypes.c_int, _p, _i64, _p, _f32, _p, _p, _p,
                                                     _i64, _p, _p, _i64, _p, _i64, _p]),
    "gnnea_gat_bwd_edge_sliced_bf16": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int,
                                                      ctypes.c_int, _p, _f32, _p, _p, _p, _i64,
                                                      _p, _p, _i64, _p, _p, _p]),
    "gnnea_gat_bwd_dst_sliced_bf16": (ctypes.c_int, [_p, _p, _i32, ctypes.c_int, ctypes.c_int,
                                                     _p, _p, _p, _p, _i64, _p, _p]),
    "gnnea_gat_fwd_sliced_range_f32": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int,
                                                      ctypes.c_int, _p, _p, _f32, _p, ctypes.c_int,
                                                      _p, _i64, _p, _p, _p, ctypes.c_int,
                                                      ctypes.c_int, ctypes.c_int, _p]),
    "gnnea_gat_fwd_sliced_range_bf16": (ctypes.c_int, [_p, _p, _i32, _p, _i64, ctypes.c_int,
                                                       ctypes.c_int, _p, _p, _f32, _p,
                                                       ctypes.c_int, _p, _i64, _p, _p, _p,
                                                       ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                       _p]),
    "gnnea_gat_bwd_src_sliced_range_f32": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int,
                                                          ctypes.c_int, _p, _i64, _i64, _p, _f32,
                                                          _p, _p, _p, _i64, _p, _p, _i64, _p,
                                                          _i64, _i64, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_int, _p]),
    "gnnea_gat_bwd_src_sliced_range_bf16": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_int,
                                                           ctypes.c_int, _p, _i64, _i64, _p, _f32,
                                                           _p, _p, _p, _i64, _p, _p, _i64, _p,
                                                           _i64, _i64, ctypes.c_int,
                                                           ctypes.c_int, ctypes.c_int, _p]),
    "gnnea_slice_pack64_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _i64, _p]),
    "gnnea_slice_pack64_bf16": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _i64, _p]),
    "gnnea_gemm_f64": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p, _i64, _p,
                                      _i64, ctypes.c_double, _p, _i64, ctypes.c_double, _p, _i64,
                                      _p]),
    "gnnea_gemm_x3t_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_gemm_x3_ws_bytes": (_i64, [_i64, _i64, _i64]),
    "gnnea_gemm_x3_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p, _i64,
                                         _p, _i64, _p, _f32, _p, _i64, _p, _i64, _p]),
    "gnnea_gemm_x3_dual_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p,
                                              _i64, _p, _i64, _p, _f32, _p, _i64, _p, _i64, _p,
                                              _i64, _p]),
    "gnnea_gemm_x3_sliced_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64, _i64, _i64, _p,
                                                _i64, _p, _i64, _p, _f32, _p, _i64, _p, _i64,
                                                _p]),
    "gnnea_sinkhorn_ws_bytes": (_i64, [ctypes.c_int, ctypes.c_int]),
    "gnnea_sinkhorn_path": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem)]),
    "gnnea_sinkhorn_init": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), _p]),
    "gnnea_sinkhorn_iterate": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), ctypes.c_int,
                                              ctypes.c_int, _p]),
    "gnnea_sinkhorn_finish": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), _p, ctypes.c_int,
                                             _i64, _p, _p, _p]),
    "gnnea_sinkhorn_shard_ws_bytes": (_i64, [ctypes.c_int, ctypes.c_int]),
    "gnnea_sinkhorn_shard_pair_len": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem)]),
    "gnnea_sinkhorn_shard_init": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), ctypes.c_int,
                                                 _p]),
    "gnnea_sinkhorn_shard_colpart": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem),
                                                    ctypes.c_int, _p, _p]),
    "gnnea_sinkhorn_shard_step": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), ctypes.c_int,
                                                 _p, ctypes.c_int, _p]),
    "gnnea_sinkhorn_shard_flag": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), _p, _p]),
    "gnnea_sinkhorn_shard_close": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), _p,
                                                  ctypes.c_int, _p]),
    "gnnea_sinkhorn_shard_finish": (ctypes.c_int, [ctypes.POINTER(SinkhornProblem), _p,
                                                   ctypes.c_int, _i64, _p, _p, _p, _p]),
    "gnnea_l1_keys_f32":(ctypes.c_int, [_p, _i64, _i32, _p, _i64, _i32, _i32, _p, _i64, _p]),
    "gnnea_l1_pairs_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i32, _i32, _p, _p]),
    "gnnea_l1_terms_f32": (ctypes.c_int, [_p, _i64, _i32, _i64, _p, _p, _p, _p]),
    "gnnea_ub_copy": (ctypes.c_int, [_p, _p, _i64, _i32, _i32, _p]),
    "gnnea_ub_gather": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _i32, _p]),
    "gnnea_l1_rank_f32": (ctypes.c_int, [_p, _i64, _i32, _p, _i64, _i32, _i32, _p, _p, _p]),
    "gnnea_l1_rank_range_f32": (ctypes.c_int, [_p, _i64, _i32, _p, _i64, _i32, _i32, _p, _i32, _p,
                                               _p]),
    "gnnea_topk_rows_f32": (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _p, _i64, _p, _i64, _i32,
                                           _i32, _p, _p, _i32, _p, _p]),
    "gnnea_margin_fwd_f32": (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                                            _p, _p, _p, _p]),
    "gnnea_margin_bwd_f32": (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                                            _p, _p, _p, _i32, _p, _p, _i32, _p, _p, _f32, _p,
                                            _i64, _p]),
    "gnnea_margin_fwd_code_f32": (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p,
                                                 _p, _p, _p, _p, _p, _i64, _p]),
    "gnnea_margin_bwd_code_f32": (ctypes.c_int, [_i32, _i32, _i32, _p, _p, _i64, _p, _p, _i32, _p,
                                                 _p, _i32, _p, _p, _f32, _p, _i64, _p]),
    "gnnea_margin_fwd_code_bf16": (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _p, _p, _p, _p, _p,
                                                  _p, _p, _p, _p, _p, _i64, _p]),
    "gnnea_margin_bwd_code_bf16": (ctypes.c_int, [_i32, _i32, _i32, _p, _p, _i64, _p, _p, _i32,
                                                  _p, _p, _i32, _p, _p, _f32, _p, _i64, _p]),
}

_LIB = None


class GnneaError(RuntimeError):
    pass


def lib():
    """Load (once) and return the native library; raise loudly when it is absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise GnneaError(
                "gnnea: native library %s is not built (run __graft_entry__.build() or "
                "`make -C gnn-mtl_amd/csrc`); there is no CPU fallback" % LIB_PATH)
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def check(rc):
    if rc != 0:
        msg = lib().gnnea_error_string(int(rc))
        raise GnneaError("gnnea call failed (%d): %s" % (rc, msg.decode() if msg else "?"))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device):
    """The caller's current HIP stream on ``device`` (the raw handle query costs ~0.2 us against
    ~3 us for building a torch Stream object: it runs once per kernel launch)."""
    if _RAW_STREAM is not None:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        return ctypes.c_void_p(_RAW_STREAM(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_SAME_DEVICE = contextlib.nullcontext()


def on_device(device):
    """torch.cuda.device(device) only when it is not already current (the common case pays no
    device switch on entry and exit)."""
    if device.index is None or device.index == torch.cuda.current_device():
        return _SAME_DEVICE
    return torch.cuda.device(device)


def require_device(*tensors):
    """The product path is HIP-only: refuse host tensors instead of silently computing on CPU."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise GnneaError(
                "gnnea: tensors must live on a HIP device (got %s); the MI355X engine has no "
                "CPU path" % t.device)
