"""The C-ABI boundary (include/cai.h <-> lib/libcai.so <-> compressai._native), on CPU.

No kernel is launched: the library is loaded, every symbol the header declares
must be exported and bound, and argument validation (which runs before any
device work) must reject bad calls with CAI_EINVAL and a message, the way the
reference's pybind layer turns std::domain_error into ValueError
(cpp_exts/ops/ops.cpp:46-64).
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cai.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cai_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def native():
    from compressai import _native

    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libcai.so not built")
    _native.lib.load()
    return _native


def test_every_declared_symbol_is_exported(native):
    raw = ctypes.CDLL(native.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(raw, f)]
    assert not missing, missing


def test_binding_table_matches_header(native):
    decl = set(declared_functions())
    bound = set(native.SIGNATURES)
    assert decl == bound, (sorted(decl - bound), sorted(bound - decl))
    assert native.lib.cai_abi_count() == len(decl)
    assert native.lib.cai_version() >= 1


def test_invalid_geometry_is_einval_with_message(native):
    lib = native.lib.load()
    g = native.ConvGeom(2, 16, 8, 8, 16, 7, 7, 5, 2, 2, 0, 0)   # 8x8 k5 s2 p2 -> 4x4, not 7x7
    rc = lib.cai_conv_fwd(ctypes.byref(g), native.BF16, None, 16, 0, None, None, 0, 0.0, None, native.BF16,
                          0, 0, 0, 0, None, 0, None)
    assert rc == native.CAI_EINVAL
    assert b"output size" in lib.cai_last_error()
    assert lib.cai_conv_packed_weight_bytes(None, native.BF16, 0) == 0


def test_conv_fwd_res_requires_residual(native):
    lib = native.lib.load()
    g = native.ConvGeom(2, 16, 8, 8, 16, 8, 8, 1, 1, 0, 0, 0)
    rc = lib.cai_conv_fwd_res(ctypes.byref(g), native.BF16, None, 16, 0, None, None, 1, 0.0, None, 16, None,
                              native.BF16, 0, 1, 0, 0, None, 0, None)
    assert rc == native.CAI_EINVAL
    assert b"null residual" in lib.cai_last_error()


def test_python_shim_raises_valueerror(native):
    g = native.ConvGeom(2, 16, 8, 8, 16, 4, 4, 9, 2, 2, 0, 0)   # kernel 9 unsupported
    with pytest.raises(ValueError, match="unsupported kernel"):
        native.lib.cai_conv_fwd(ctypes.byref(g), native.BF16, None, 16, 0, None, None, 0, 0.0, None, native.BF16,
                                0, 0, 0, 0, None, 0, None)


def test_small_deconv_gate(native):
    lib = native.lib.load()
    ok = native.ConvGeom(2, 128, 16, 16, 3, 32, 32, 5, 2, 2, 1, 1)
    wide = native.ConvGeom(2, 128, 16, 16, 32, 32, 32, 5, 2, 2, 1, 1)
    assert lib.cai_deconv_small_workspace_bytes(ctypes.byref(ok), native.BF16) > 0
    assert lib.cai_deconv_small_workspace_bytes(ctypes.byref(wide), native.BF16) == 0


def test_gdn_channel_counts_validated(native):
    with pytest.raises(ValueError):
        native.lib.cai_gdn_fwd(native.BF16, None, 48, 16, 48, None, None, 0, None, 48, None)


def test_product_path_has_no_cpu_fallback():
    """A CPU tensor must be refused, not silently computed by torch."""
    import torch

    from compressai.layers import Conv2d

    m = Conv2d(8, 8, 3, padding=1)
    with pytest.raises((RuntimeError, ValueError)):
        m(torch.zeros(1, 8, 8, 8))


def test_empty_conv_output_is_einval(native):
    """A kernel larger than its (padded) input is rejected before any launch sizing."""
    lib = native.lib.load()
    g = native.ConvGeom(1, 16, 3, 3, 16, -1, -1, 5, 1, 0, 0, 0)
    assert lib.cai_conv_workspace_bytes(ctypes.byref(g), native.BF16, 0) == 0
    with pytest.raises(ValueError, match="empty output"):
        native.lib.cai_conv_fwd(ctypes.byref(g), native.BF16, None, 16, 0, None, None, 0, 0.0, None, native.BF16,
                                0, 0, 0, 0, None, 0, None)


def test_edge_gate(native):
    """csrc/edge.hip takes stride-2, k odd <= 5, pad k/2 image-side layers with <= 3 image channels,
    128/192 feature channels, bf16 only."""
    lib = native.lib.load()
    G = native.ConvGeom
    yes = [G(2, 3, 256, 256, 128, 128, 128, 5, 2, 2, 0, 0), G(2, 128, 16, 16, 3, 32, 32, 5, 2, 2, 1, 1),
           G(1, 1, 64, 64, 192, 32, 32, 3, 2, 1, 0, 0), G(1, 192, 8, 9, 2, 16, 18, 3, 2, 1, 1, 1)]
    no = [G(2, 4, 64, 64, 128, 32, 32, 5, 2, 2, 0, 0),     # 4 image channels
          G(2, 3, 64, 64, 64, 32, 32, 5, 2, 2, 0, 0),      # 64 feature channels
          G(2, 3, 63, 64, 128, 32, 32, 5, 2, 2, 0, 0),     # odd image height
          G(2, 128, 16, 16, 3, 16, 16, 5, 1, 2, 0, 1),     # stride 1
          G(2, 3, 64, 64, 128, 32, 32, 4, 2, 1, 0, 0)]     # even kernel
    for g in yes:
        assert lib.cai_edge_supported(ctypes.byref(g), native.BF16) == 1
        assert lib.cai_edge_workspace_bytes(ctypes.byref(g), native.BF16) > 0
        assert lib.cai_edge_supported(ctypes.byref(g), native.F32) == 0
    for g in no:
        assert lib.cai_edge_supported(ctypes.byref(g), native.BF16) == 0
        assert lib.cai_edge_workspace_bytes(ctypes.byref(g), native.BF16) == 0
    with pytest.raises(ValueError, match="unsupported geometry"):
        native.lib.cai_edge_conv_fwd(ctypes.byref(no[0]), None, None, None, None, 128, None)


def test_halo_kernel_selection(native):
    """Host-side kernel choice (no launch): the halo-staged stride-1 k3 kernel takes both directions of
    3x3 s1 p1 convs with 64-multiple input channels on >= 8 x 32 outputs (192-channel tiles for 192/384/768
    output channels), and the s^2-phase kernel's 192-channel tiles take the k5 s2 transposed direction at N = 192
    (test_kernels_gpu.py CONV_CASES runs these geometries on the GPU)."""
    lib = native.lib.load()
    G = native.ConvGeom

    def name(g, d):
        return lib.cai_conv_kernel_name(ctypes.byref(g), native.BF16, d, 0).decode()

    assert name(G(4, 192, 128, 128, 192, 128, 128, 3, 1, 1, 0, 0), 0) == "conv_halo_s1_kernel<192>"
    assert name(G(4, 192, 128, 128, 192, 128, 128, 3, 1, 1, 0, 0), 1) == "conv_halo_s1_kernel<192>"
    assert name(G(4, 192, 64, 64, 768, 64, 64, 3, 1, 1, 0, 0), 0) == "conv_halo_s1_kernel<192>"
    # its input gradient (768 -> 192, 64 tiles): K split four ways on the halo kernel
    assert name(G(4, 192, 64, 64, 768, 64, 64, 3, 1, 1, 0, 0), 1) == "conv_halo_s1_kernel<192>"
    assert name(G(4, 128, 64, 128, 96, 64, 128, 3, 1, 1, 0, 0), 0) == "conv_halo_s1_kernel<128>"
    assert name(G(4, 128, 64, 64, 256, 64, 64, 3, 1, 1, 0, 0), 0) == "conv_halo_s1_kernel<128>"
    assert name(G(4, 96, 64, 128, 128, 64, 128, 3, 1, 1, 0, 0), 0) != "conv_halo_s1_kernel<128>"   # Cin % 64
    assert "halo" not in name(G(16, 192, 16, 16, 192, 16, 16, 3, 1, 1, 0, 0), 0)                 # 16 wide
    assert name(G(16, 192, 64, 64, 192, 128, 128, 5, 2, 2, 1, 1), 0) == "conv_halo_phase_kernel<192>"
    assert name(G(16, 192, 128, 128, 192, 64, 64, 5, 2, 2, 0, 0), 1) == "conv_halo_phase_kernel<192>"
    assert name(G(8, 64, 64, 64, 192, 128, 128, 5, 2, 2, 1, 1), 0) == "conv_halo_phase_kernel<192>"
    assert name(G(8, 192, 128, 128, 64, 64, 64, 5, 2, 2, 0, 0), 1) == "conv_halo_phase_kernel<192>"
    assert "halo" not in name(G(16, 192, 32, 32, 192, 64, 64, 5, 2, 2, 1, 1), 0)    # 256 blocks
    # 128 channels: the four-phase kernel from 256 tiles (one block per CU), the per-phase kernel below
    assert name(G(16, 128, 64, 64, 128, 128, 128, 5, 2, 2, 1, 1), 0) == "conv_halo_quad_kernel"
    assert name(G(16, 128, 128, 128, 128, 64, 64, 5, 2, 2, 0, 0), 1) == "conv_halo_quad_kernel"
    assert name(G(8, 128, 64, 64, 128, 128, 128, 5, 2, 2, 1, 1), 0) == "conv_halo_phase_kernel"
    assert name(G(16, 128, 32, 32, 128, 64, 64, 5, 2, 2, 1, 1), 0) == "conv_halo_phase_kernel"
    assert name(G(16, 192, 64, 64, 128, 128, 128, 5, 2, 2, 1, 1), 0) == "conv_halo_phase_kernel"   # Cin 192
    # weight gradient: the halo-staged kernel's stride-1 form for 64-multiple G widths
    if os.environ.get("CAI_HALO_WGRAD_S1_OFF", "0") in ("", "0"):
        assert name(G(4, 192, 128, 128, 192, 128, 128, 3, 1, 1, 0, 0), 2) == "wgrad_halo_kernel<3,s1>"
        assert name(G(2, 64, 512, 640, 64, 512, 640, 3, 1, 1, 0, 0), 2) == "wgrad_halo_kernel<3,s1>"
    assert "halo" not in name(G(4, 192, 32, 32, 192, 32, 32, 3, 1, 1, 0, 0), 2)
    # the stride-1 conv kernel needs >= 128 tiles (64x64 at B = 4: 64 tiles, conv_glds_kernel)
    assert "halo" not in name(G(4, 192, 64, 64, 192, 64, 64, 3, 1, 1, 0, 0), 0)
    assert lib.cai_conv_kernel_name(ctypes.byref(G(4, 192, 128, 128, 192, 128, 128, 3, 1, 1, 0, 0)), native.F32,
                                    0, 0).decode().startswith("conv_gemm")
