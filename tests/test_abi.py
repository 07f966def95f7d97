"""The C-ABI library loads and exports every symbol include/gnnea.h declares (no GPU needed)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gnnea.h")
HOST_HEADER = os.path.join(ROOT, "include", "gnnea_host.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\*?\s+\*?(gnnea_[a-z0-9_]+)\s*\(", src, re.M)
    return sorted(set(names))


def test_header_declares_the_hot_path():
    names = declared_functions()
    for must in ("gnnea_coo_to_csr", "gnnea_spmm_csr_f32", "gnnea_spmm_highway_f32",
                 "gnnea_gat_fwd_f32", "gnnea_gat_bwd_prep_f32", "gnnea_gat_bwd_src_f32",
                 "gnnea_gat_bwd_dst_f32", "gnnea_spmm_csr_beta_f32", "gnnea_perm_invert",
                 "gnnea_gemm_f32", "gnnea_sinkhorn_iterate", "gnnea_sinkhorn_finish",
                 "gnnea_l1_keys_f32", "gnnea_topk_rows_f32", "gnnea_l1_rank_f32",
                 "gnnea_l1_pairs_f32", "gnnea_margin_fwd_f32", "gnnea_margin_bwd_f32",
                 "gnnea_spmm_csr_bf16", "gnnea_spmm_highway_bf16", "gnnea_act_bwd_bf16",
                 "gnnea_highway_bwd_bf16", "gnnea_highway_bwd_ld_f32", "gnnea_highway_bwd_ld_bf16", "gnnea_gemm_bf16", "gnnea_gat_scores_bf16",
                 "gnnea_gat_fwd_bf16", "gnnea_gat_bwd_prep_bf16", "gnnea_gat_bwd_src_bf16",
                 "gnnea_gat_bwd_dst_bf16", "gnnea_spmm_sliced_f32", "gnnea_slice_pack_f32",
                 "gnnea_act_bwd_sliced_f32", "gnnea_gemm_sliced_f32",
                 "gnnea_margin_fwd_code_f32", "gnnea_margin_bwd_code_f32"):
        assert must in names


def test_host_library_exports_every_declared_symbol():
    from gnnea import ingest
    if not os.path.exists(ingest.LIB_PATH):
        pytest.skip("libgnnea_host.so not built")
    names = declared_functions(HOST_HEADER)
    assert {"gnnea_h_loadfile", "gnnea_h_adjacency", "gnnea_h_relation_groups"} <= set(names)
    L = ingest.lib()
    for name in names:
        assert hasattr(L, name) and name in ingest.SIGNATURES, name
    out = subprocess.run(["nm", "-D", "--defined-only", ingest.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert set(names) <= set(re.findall(r" T (gnnea_\w+)", out))


def test_library_exports_every_declared_symbol():
    from gnnea import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgnnea.so not built")
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, "ctypes signature missing for " + name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (gnnea_\w+)", out))
    assert set(declared_functions()) <= exported


def test_host_only_entry_points():
    from gnnea import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgnnea.so not built")
    L = _lib.lib()
    assert L.gnnea_abi_version() == 1
    assert b"workspace" in L.gnnea_error_string(-2)
    assert L.gnnea_sinkhorn_ws_bytes(3000, 3000) > 3000 * 8 * 4
    assert L.gnnea_gemm_ws_bytes(300, 300, 2_000_000) > 0
    # argument validation never touches the device
    assert L.gnnea_spmm_csr_f32(None, None, None, -1, 300, None, 300, None, 300, 1, None) == -1
    assert L.gnnea_gemm_f32(0, 0, 4, 4, 4, None, 4, None, 4, None, 0.0, None, 4, None, 0,
                            None) == -1
    # slice-major entry points: D % 4, slice stride and alignment are checked on the host
    assert L.gnnea_spmm_sliced_f32(None, None, None, -1, 300, None, 64, None, 300, 1, None) == -1
    assert L.gnnea_spmm_sliced_f32(16, 16, 16, 4, 30, 16, 64 * 4, 16, 32, 1, None) == -1
    assert L.gnnea_slice_pack_f32(16, 300, 10, 300, 16, 63, None) == -1
    assert L.gnnea_act_bwd_sliced_f32(16, 300, 16, 300, 10, 302, 1, 16, 640, None) == -1
    assert L.gnnea_gemm_sliced_f32(0, 1, 10, 300, 8, 16, 8, 16, 8, None, 0.0, 16, 66, None, 0,
                                   None) == -1


def test_sliced_gat_refuses_three_heads_per_slice():
    """The sliced GAT kernels keep two heads per 64-column slice: d_head = 40 (slice 1 = heads
    1, 2, 3) is refused by every sliced entry point on the host, before any launch; the Python
    gate (ops.gat_two_heads_per_slice) agrees, so that shape takes the row-major passes."""
    from gnnea import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgnnea.so not built")
    L = _lib.lib()
    for heads, dh, ok in ((4, 40, False), (4, 36, False), (2, 50, True), (8, 40, False), (4, 75, True),
                          (8, 32, True), (3, 48, True), (1, 300, True), (2, 64, True),
                          (4, 31, False)):
        assert ops.gat_two_heads_per_slice(heads, dh) == ok, (heads, dh)
        if ok:
            continue
        for fn in (L.gnnea_gat_fwd_sliced_f32, L.gnnea_gat_fwd_sliced_bf16):
            assert fn(16, 16, 4, 16, 64 * 4, heads, dh, 16, 16, 0.2, None, 1, 16, heads * dh,
                      16, 16, 16, None) == -1
        for fn in (L.gnnea_gat_bwd_prep_sliced_f32, L.gnnea_gat_bwd_prep_sliced_bf16):
            assert fn(4, heads, dh, 16, 16, heads * dh, 16, 16, 16, 1, 16, 256, 16, None) == -1
        for fn in (L.gnnea_gat_bwd_src_sliced_f32, L.gnnea_gat_bwd_src_sliced_bf16):
            assert fn(16, 16, None, 4, heads, dh, 16, heads * dh, 16, 0.2, None, 16, 16, 256, 16,
                      16, 4, 16, heads * dh, None) == -1
        for fn in (L.gnnea_gat_bwd_edge_sliced_f32, L.gnnea_gat_bwd_edge_sliced_bf16):
            assert fn(16, 16, None, 4, heads, dh, 16, 0.2, None, 16, 16, 4, 16, None, 0, 16, 16,
                      None) == -1
        for fn in (L.gnnea_gat_bwd_dst_sliced_f32, L.gnnea_gat_bwd_dst_sliced_bf16):
            assert fn(16, 16, 4, heads, dh, 16, 16, None, 16, heads * dh, 16, None) == -1
    # the 64-column pack: slice stride and width checked on the host
    assert L.gnnea_slice_pack64_bf16(16, 300, 10, 300, 16, 63, None) == -1
    assert L.gnnea_slice_pack64_f32(16, 302, 10, 302, 16, 640, None) == -1
