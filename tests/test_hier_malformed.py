"""Malformed hierarchy files are refused with HLGS_ERR_ARG before anything is sized from their headers.

The reference's loader (gaussianhierarchy/hierarchy_loader.cpp:26-189) trusts the counts in the header; here every
count is checked against the file's size first (csrc/hier_io.cpp hlgs_hier_info_read): truncated files, negative
Gaussian or node counts, an SH degree out of range and a node count beyond the file all return an error, never a read
past the buffers.  tests/test_sanitizers.py runs this file against the ASan + UBSan build of the same host code.
"""
import os

import numpy as np
import pytest
import torch

from oracle import hier_format as HF

ERR_ARG = 1  # HLGS_ERR_ARG (include/hlgs.h)


def _lib():
    from hlgs_core import _lib as L
    return L.load()


def _info(path, dynamic):
    from hlgs_core import _lib as L
    info = L.HierInfo()
    rc = _lib().hlgs_hier_info_read(str(path).encode(), int(dynamic), L.C.byref(info))
    return rc, info


def _dhier(tmp_path, G=40, deg=2):
    rng = np.random.default_rng(G + deg)
    f = np.float32
    nodes = np.zeros((G, 6), np.int32)
    nodes[:, 1] = -1
    p = tmp_path / f"ok_{G}_{deg}.dhier"
    HF.write_dhier(str(p), rng.normal(size=(G, 3)).astype(f), rng.normal(size=(G, 16, 3)).astype(f),
                   rng.uniform(size=(G, 1)).astype(f), rng.normal(size=(G, 3)).astype(f),
                   rng.normal(size=(G, 4)).astype(f), nodes, deg)
    return p


def _hier(tmp_path, compressed, P=30, N=5):
    rng = np.random.default_rng(7)
    f = np.float32
    nodes = np.zeros((N, 7), np.int32)
    nodes[:, 1] = -1
    p = tmp_path / f"ok_{int(compressed)}.hier"
    HF.write_hier(str(p), rng.normal(size=(P, 3)).astype(f), rng.normal(size=(P, 16, 3)).astype(f),
                  rng.uniform(size=(P, 1)).astype(f), rng.normal(size=(P, 3)).astype(f),
                  rng.normal(size=(P, 4)).astype(f), nodes, rng.normal(size=(N, 2, 4)).astype(f), compressed=compressed)
    return p


def _write(path, data):
    with open(path, "wb") as fh:
        fh.write(data)
    return path


def test_valid_files_are_accepted(tmp_path):
    rc, info = _info(_dhier(tmp_path), True)
    assert rc == 0 and info.G == 40 and info.sh_degree == 2 and info.N == 40
    for c in (False, True):
        rc, info = _info(_hier(tmp_path, c), False)
        assert rc == 0 and info.G == 30 and info.N == 5


@pytest.mark.parametrize("cut", [0, 2, 4, 7, 8, 100, -4, -1])
def test_truncated_dhier(tmp_path, cut):
    b = open(_dhier(tmp_path), "rb").read()
    p = _write(tmp_path / "t.dhier", b[:cut] if cut >= 0 else b[:len(b) + cut])
    assert _info(p, True)[0] == ERR_ARG


@pytest.mark.parametrize("compressed", [False, True])
@pytest.mark.parametrize("frac", [0.0, 0.001, 0.3, 0.9, 0.999])
def test_truncated_hier(tmp_path, compressed, frac):
    b = open(_hier(tmp_path, compressed), "rb").read()
    p = _write(tmp_path / "t.hier", b[:int(len(b) * frac)])
    assert _info(p, False)[0] == ERR_ARG


def test_dhier_bad_header_counts(tmp_path):
    b = bytearray(open(_dhier(tmp_path), "rb").read())
    for G, deg in ((-1, 2), (-2 ** 31, 2), (40, -1), (40, 4), (40, 2 ** 30), (41, 2), (2 ** 31 - 1, 3)):
        c = bytearray(b)
        c[0:8] = np.array([G, deg], np.int32).tobytes()
        assert _info(_write(tmp_path / "h.dhier", bytes(c)), True)[0] == ERR_ARG, (G, deg)


@pytest.mark.parametrize("compressed", [False, True])
def test_hier_bad_node_count(tmp_path, compressed):
    P, N = 30, 5
    b = bytearray(open(_hier(tmp_path, compressed, P, N), "rb").read())
    per = 12 + 2 * (4 + 3 + 1 + 48) if compressed else 12 + 16 + 12 + 4 + 4 * 48
    off = 4 + P * per
    assert np.frombuffer(bytes(b[off:off + 4]), np.int32)[0] == N
    for n in (-1, -2 ** 31, N + 1, 2 ** 31 - 1):
        c = bytearray(b)
        c[off:off + 4] = np.array([n], np.int32).tobytes()
        assert _info(_write(tmp_path / "n.hier", bytes(c)), False)[0] == ERR_ARG, n
    for g in (P + 1, 2 ** 31 - 1, -(2 ** 31)):  # a Gaussian count beyond the file (either layout's sign)
        c = bytearray(b)
        c[0:4] = np.array([g], np.int32).tobytes()
        assert _info(_write(tmp_path / "g.hier", bytes(c)), False)[0] == ERR_ARG, g


def test_loaders_raise_on_malformed_files(tmp_path):
    """The Python loaders (gaussian_hierarchy._C) turn the error into an exception instead of sizing tensors."""
    import gaussian_hierarchy as GH
    b = open(_dhier(tmp_path), "rb").read()
    with pytest.raises(RuntimeError, match="truncated"):
        GH.load_dynamic_hierarchy(str(_write(tmp_path / "x.dhier", b[:len(b) // 2])))
    hb = bytearray(open(_hier(tmp_path, True), "rb").read())
    off = 4 + 30 * (12 + 2 * 56)
    hb[off:off + 4] = np.array([-7], np.int32).tobytes()
    with pytest.raises(RuntimeError, match="negative node count"):
        GH.load_hierarchy(str(_write(tmp_path / "x.hier", bytes(hb))))


def test_expand_to_target_rejects_bad_child_links():
    from hlgs_core import _lib as L
    nodes = np.zeros((3, 7), np.int32)
    nodes[0, 0], nodes[0, 5], nodes[0, 6] = 2, 1, 5  # five children from index 1: past the node array
    cnt = L.C.c_int(0)
    out = np.zeros(16, np.int32)
    rc = _lib().hlgs_expand_to_target(3, nodes.ctypes.data_as(L.C.c_void_p), 0, out.ctypes.data_as(L.C.c_void_p), 16,
                                      L.C.byref(cnt))
    assert rc == ERR_ARG


def test_spt_build_rejects_bad_links():
    from hlgs_core import spt
    G = 8
    nodes = torch.zeros(G, 6, dtype=torch.int32)
    nodes[:, 1] = -1
    nodes[0, 2], nodes[0, 3] = 2, 50  # first child out of range
    xyz = torch.zeros(G, 3)
    sc = torch.zeros(G, 3) + 3.0
    with pytest.raises(RuntimeError, match="out of range"):
        spt.build_hierarchical_spt(nodes, xyz, sc, 0, 1e-3, 0.1)
