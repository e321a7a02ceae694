"""The C-ABI library: loads, exports every symbol include/anr.h declares, validates
arguments host-side. No kernel launches (CPU only)."""

import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "anr.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(anr_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from atmonr_amd import _lib

    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 18
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, f"not exported: {missing}"
    # the Python binding declares exactly the header's functions
    assert sorted(_lib.symbols()) == declared


def test_abi_version_and_struct_sizes():
    from atmonr_amd import _lib

    assert _lib.load().anr_abi_version() == 5
    # __graft_entry__.build() checks the built library against the header's define
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                       "anr.h")
    with open(hdr) as f:
        want = next(int(ln.split()[2]) for ln in f if ln.startswith("#define ANR_ABI_VERSION"))
    assert want == _lib.load().anr_abi_version()
    assert ctypes.sizeof(_lib.PrepParams) == 96
    assert ctypes.sizeof(_lib.MlpDesc) == 32


def test_hashgrid_init_matches_oracle():
    from atmonr_amd import _lib
    from oracle import ref_tcnn

    for cfg in [(3, 16, 16, 1.3819, 21), (3, 16, 16, 1.3819, 19), (2, 16, 16, 1.3819, 19),
                (3, 8, 4, 2.0, 12)]:
        d = _lib.hashgrid_desc(cfg[0], cfg[1], 2, cfg[2], cfg[3], cfg[4])
        offs, sizes, res, scales, entries = ref_tcnn.grid_levels(*cfg)
        assert d.n_params == 2 * entries
        assert list(d.offsets)[: cfg[1]] == offs.tolist()
        assert list(d.resolutions)[: cfg[1]] == res.tolist()
        assert list(d.scales)[: cfg[1]] == pytest.approx(scales.tolist(), rel=1e-7)


def test_invalid_arguments_report_errors():
    from atmonr_amd import _lib

    with pytest.raises(_lib.ANRError, match="n_dims"):
        _lib.hashgrid_desc(4, 16, 2, 16, 1.38, 19)
    with pytest.raises(_lib.ANRError, match="width"):
        _lib.mlp_desc(32, 16, 48, 1, False)
    lib = _lib.load()
    rc = lib.anr_hashgrid_fwd(None, None, 3, 10, None, 0, None, 0, 32, None)
    assert rc == -1 and b"null" in lib.anr_last_error()
    # a zero-size call is a no-op success even without device pointers for outputs
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    assert lib.anr_hashgrid_fwd(ctypes.byref(d), 1, 3, 0, 1, 1, 1, 1, 32, None) == 0


def test_mlp_param_counts():
    from atmonr_amd import _lib

    lib = _lib.load()
    for n_in, n_out, w, h, expect in [(32, 16, 32, 1, 32 * 32 + 16 * 32),
                                      (19, 4, 32, 2, 32 * 32 + 32 * 32 + 16 * 32),
                                      (36, 4, 64, 2, 64 * 48 + 64 * 64 + 16 * 64)]:
        d = _lib.mlp_desc(n_in, n_out, w, h, False)
        assert lib.anr_mlp_n_params(ctypes.byref(d)) == expect
        # backward workspace: one dW row per wavefront (16-row tiles, 4 per block), only
        # for batches up to 64Ki rows
        nw = (8192 + 15) // 16 + 3
        assert lib.anr_mlp_bwd_workspace_bytes(ctypes.byref(d), 8192) == 4 * nw * expect
        assert lib.anr_mlp_bwd_workspace_bytes(ctypes.byref(d), 1 << 17) == 0
        assert lib.anr_mlp_bwd_workspace_bytes(ctypes.byref(d), 0) == 0


def test_hash_bwd_chunk_rule_is_queried_from_the_library():
    """tools/hash_requests.py replays the hash backward's chunking on the CPU (the
    by-cause request analysis, and the reference for the GPU count instrument's test);
    the chunk length comes from the library itself, so the replay cannot drift from the
    kernel's rule (r04: a stale Python copy of the rule once counted 512-sample chunks
    while the kernel ran 256)."""
    from atmonr_amd import _lib
    from tools import hash_requests

    lib = _lib.load()
    for M, K in [(0, 0), (1, 1), (4096, 1), (1024 * 1024, 256), (8192 * 1024, 256),
                 (100_000, 24)]:
        assert lib.anr_hashgrid_bwd_chunk(M) == K, M
        if M:
            assert hash_requests.bwd_chunk(M) == K
