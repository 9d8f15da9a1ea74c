"""C-ABI library checks that need no GPU: the shared library loads and exports
every entry point include/gtf.h declares; the ctypes structs match the header."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "gtf.h")


def _declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(gtf_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from gtf import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libgtf.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gtf_\w+)", out))
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    assert set(_native.SYMBOLS) <= exported


def test_library_loads_and_binds():
    from gtf import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libgtf.so not built")
    L = _native.lib()
    assert L.gtf_version().decode().startswith("gtf")
    # workspace size is a pure host function
    assert L.gtf_workspace_bytes(100, 1000) >= 256 + 8 * 1000
    # tag-propagation workspace: counters, keep [E], processed [N], the second tag array [N]
    assert L.gtf_tag_workspace_bytes(100, 1000) >= 8 + 1000 + 100 + 8 * 100
    assert L.gtf_tag_workspace_bytes(0, 0) > 0


def test_struct_layout_matches_header():
    """compile a tiny C probe of offsetof()/sizeof() of every field of every struct
    against the header and compare with the ctypes mirrors"""
    from gtf import _native as nat
    py = {"gtf_graph": nat.GtfGraph, "gtf_nodes": nat.GtfNodes, "gtf_states": nat.GtfStates,
          "gtf_edges": nat.GtfEdges, "gtf_params": nat.GtfParams, "gtf_kl_graph": nat.GtfKlGraph, "gtf_tse_extra": nat.GtfTseExtra, "gtf_shard": nat.GtfShard, "gtf_halo": nat.GtfHalo,
          "gtf_extract_params": nat.GtfExtractParams, "gtf_extract_io": nat.GtfExtractIO,
          "gtf_kl_out": nat.GtfKlOut, "gtf_event_csr": nat.GtfEventCsr,
          "gtf_candidate_graph": nat.GtfCandidateGraph, "gtf_pair_out": nat.GtfPairOut,
          "gtf_diag": nat.GtfDiag}
    lines = []
    for t, cls in py.items():
        lines += ['  printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (t, f, t, f) for f, _ in cls._fields_]
        lines.append('  printf("sizeof.%s %%zu\\n", sizeof(%s));' % (t, t))
    probe = "#include <stdio.h>\n#include <stddef.h>\n#include \"gtf.h\"\nint main(void) {\n%s\n  return 0;\n}\n" % \
        "\n".join(lines)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.check_call(["gcc", "-I", os.path.dirname(HDR), c, "-o", exe])
        got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([exe], text=True).split("\n") if l)
    assert len(got) == sum(len(c._fields_) + 1 for c in py.values())
    for k, v in got.items():
        t, f = k.split(".")
        if t == "sizeof":
            assert ctypes.sizeof(py[f]) == int(v), k
        else:
            assert getattr(py[t], f).offset == int(v), k


def test_no_fallback_without_library(monkeypatch, tmp_path):
    """the product path fails loudly when the HIP library is missing"""
    from gtf import _native
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_native, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _native.lib()


def test_graph_struct_carries_abi_version():
    """gtf_graph starts with its size and GTF_ABI_VERSION; the ctypes mirror fills both"""
    from gtf import _native as nat
    ver = re.search(r"#define GTF_ABI_VERSION (\d+)u", open(HDR).read())
    assert ver and int(ver.group(1)) == nat.ABI_VERSION
    g = nat.GtfGraph(n_nodes=3)
    assert g.struct_size == ctypes.sizeof(nat.GtfGraph) and g.abi_version == nat.ABI_VERSION
    assert nat.GtfGraph.struct_size.offset == 0 and nat.GtfGraph.abi_version.offset == 4


def test_abi_mismatch_is_refused_without_a_gpu():
    """a gtf_graph of another layout is refused (-3) before any device work"""
    from gtf import _native as nat
    if not os.path.exists(nat.LIB_PATH):
        pytest.skip("libgtf.so not built")
    L = nat.lib()
    g = nat.GtfGraph(n_nodes=0)
    g.abi_version = nat.ABI_VERSION + 1
    cnt = ctypes.c_int64(0)
    z = ctypes.c_void_p(0)
    rc = L.gtf_updated_state_pair_counts(ctypes.byref(g), ctypes.byref(nat.GtfNodes()), ctypes.byref(nat.GtfStates()),
                                         ctypes.byref(nat.GtfEdges()), ctypes.byref(cnt), z)
    assert rc == -3 and b"ABI mismatch" in L.gtf_last_error()


def test_kl_gnn_stride_is_checked_without_a_gpu():
    """gtf_parabolic_kl refuses a gnn_stride other than 0, 2 or 4 (-2) before any device work"""
    from gtf import _native as nat
    if not os.path.exists(nat.LIB_PATH):
        pytest.skip("libgtf.so not built")
    L = nat.lib()
    g = nat.GtfKlGraph(n_nodes=0, n_slots=0, gnn_stride=3)
    rc = L.gtf_parabolic_kl(ctypes.byref(g), 0, ctypes.byref(nat.GtfKlOut()), ctypes.c_void_p(0))
    assert rc == -2 and b"gnn_stride" in L.gtf_last_error()


def test_rccl_is_loaded_lazily():
    """libgtf links no RCCL (gtf_comm_* dlopen it on first use): the drop-in CLIs that never
    touch a collective do not map its ~0.5 GB of device code at start-up"""
    from gtf import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libgtf.so not built")
    out = subprocess.run(["readelf", "-d", _native.LIB_PATH], capture_output=True, text=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)
    assert needed and not any("rccl" in n for n in needed), needed
    L = _native.lib()
    comm = ctypes.c_void_p()
    assert L.gtf_comm_init(ctypes.byref(comm), 0, 0, None) != 0      # bad arguments, no RCCL needed
    assert b"bad arguments" in L.gtf_last_error()
