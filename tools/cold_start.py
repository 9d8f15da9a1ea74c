"""Where a drop-in CLI invocation's wall time goes (GPU box): every probe runs in a fresh
child process (this parent never touches the GPU), three times each.

  python tools/cold_start.py OUT.json

probes: interpreter alone; the drop-in modules' imports; import torch; torch + its first
device tensor; the HIP runtime through ctypes (hipInit, one allocation, copy, sync);
libgtf.so loaded first and its error-word calls; DeviceGraph (torch) on a tiny event with its
first extrapolation (code-object load); the extrapolation CLI
itself on the vol-7 full-load directory (bench.dropin_input_vol7)."""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnn-track-finding_amd")

HIP = r"""
import ctypes, numpy as np
h = ctypes.CDLL('libamdhip64.so.7')
assert h.hipInit(0) == 0 and h.hipSetDevice(0) == 0
p = ctypes.c_void_p()
assert h.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)) == 0
a = np.ones(1 << 17)
assert h.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1) == 0
assert h.hipDeviceSynchronize() == 0
"""

GTF = r"""
import ctypes, numpy as np
g = ctypes.CDLL(%r)                  # libgtf first: its NEEDED libamdhip64.so.7 is the runtime
h = ctypes.CDLL('libamdhip64.so.7')  # the same, already loaded
P = ctypes.c_void_p
g.gtf_clear_errors.argtypes = [P, P]
g.gtf_read_errors.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P]
assert h.hipInit(0) == 0 and h.hipSetDevice(0) == 0
ws = ctypes.c_void_p()
assert h.hipMalloc(ctypes.byref(ws), ctypes.c_size_t(1 << 16)) == 0
assert g.gtf_clear_errors(ws, None) == 0
f = ctypes.c_uint32(1)
assert g.gtf_read_errors(ws, ctypes.byref(f), None) == 0 and f.value == 0
""" % os.path.join(PKG, "gtf", "libgtf.so")

PROBES = [
    ("interpreter", "pass"),
    ("dropin_imports", "import sys; sys.path.insert(0, %r); from gtf import stages, dropin, params" % PKG),
    ("import_torch", "import torch"),
    ("torch_first_tensor", "import torch; x = torch.ones(1 << 17, device='cuda'); torch.cuda.synchronize()"),
    ("hip_ctypes", HIP),
    ("hip_ctypes_libgtf_load", GTF),
    ("torch_devicegraph_first_extrapolate",
     "import sys; sys.path.insert(0, %r); from gtf import synth, device; from gtf.params import Params; "
     "d = device.DeviceGraph(synth.workload('tiny50')); d.extrapolate(Params()); d.torch.cuda.synchronize()" % PKG),
]


def timed(cmd, env=None):
    t = time.perf_counter()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    dt = time.perf_counter() - t
    if r.returncode:
        raise RuntimeError("%s failed (%d): %s" % (cmd[:3], r.returncode, r.stderr[-2000:]))
    return dt


def main(out):
    res = {}
    for name, code in PROBES:
        res[name] = [timed([sys.executable, "-c", code]) for _ in range(3)]
        print(name, ["%.3f" % x for x in res[name]], flush=True)
    sys.path[:0] = [ROOT, PKG]
    import bench
    from gtf import stages as st
    from gtf.params import Params
    p = Params()
    tmp = tempfile.mkdtemp()
    try:
        ind = os.path.join(tmp, "in") + "/"
        os.makedirs(ind)
        for i, s in enumerate(bench.dropin_input_vol7(p)):
            st.save_network(ind, i, s)
        cli = os.path.join(PKG, "extrapolate", "extrapolate_merged_states.py")
        runs = []
        for r in range(3):
            outd = os.path.join(tmp, "out%d" % r) + "/"
            os.makedirs(outd)
            runs.append(timed([sys.executable, cli, "-i", ind, "-o", outd, "-c", "2.0", "-e", "0.3", "-z", "0.4",
                               "-m", "0.6", "-b", "550"]))
            print("cli_extrapolate", "%.3f" % runs[-1], flush=True)
        res["cli_extrapolate_vol7"] = runs
    finally:
        shutil.rmtree(tmp)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
