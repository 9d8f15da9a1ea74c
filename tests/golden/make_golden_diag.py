"""Golden fixture for the diagnostics outputs (SURVEY §5 "Metrics / logging"): the truth-based
outlier-masking counts the REFERENCE's stages print, captured from its own stdout.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_diag.py       # writes tests/golden/diag_vol7.json

On make_golden.py's volume-7 network subset (the inputs of cluster_tse.npz,
extrapolate_it2.npz and update_it2.npz) it runs, with stdout captured:

* clustering on track_state_estimates (-c 1.0 -k 2.0): the block printed after the
  subgraph loop (clustering.py:342-369);
* the extrapolation stage body: message_passing (extrapolate_merged_states.py:496-518),
  then reweight twice (helper.py:203-225);
* the update stage (remove_state_metadata.py via its CLI): its reweight.

Each printed block gives (numerator, denominator) and, when the denominator is non-zero,
tp / fp / tn / fn. The node truth ids of the subset are stored with them (the packed
fixtures do not carry truth).
"""
import io
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as M  # noqa: E402

h = M.h


def parse(text):
    """the confusion blocks of one captured stage output, in print order"""
    blocks = []
    for m in re.finditer(r"numerator: (\S+) denominator: (\S+)", text):
        blocks.append({"numerator": int(m.group(1)), "denominator": int(m.group(2))})
    tps = re.findall(r"true positive number:\s+(\S+)\s+false positive number:\s+(\S+)", text)
    tns = re.findall(r"true negative number:\s+(\S+)\s+false negative number:\s+(\S+)", text)
    j = 0
    for b in blocks:
        if b["denominator"] != 0:
            b.update(tp=int(tps[j][0]), fp=int(tps[j][1]), tn=int(tns[j][0]), fn=int(tns[j][1]))
            j += 1
    return blocks


class Capture:
    def __enter__(self):
        self._o = sys.stdout
        self.buf = io.StringIO()
        sys.stdout = self.buf
        return self

    def __exit__(self, *a):
        sys.stdout = self._o


def main():
    with M._Quiet():
        net0 = M.build_network()
    order = sorted(range(len(net0)), key=lambda i: -len(net0[i]))   # make_golden.main's subset
    keep = set(order[:1])
    tot = 0
    for i in range(len(net0)):
        if tot > 3000:
            break
        keep.add(i)
        tot += len(net0[i])
    net = [net0[i] for i in sorted(keep)]
    truth = {int(n): int(s.nodes[n]["truth_particle"]) for s in net for n in s.nodes}
    out = {"truth": truth}

    class _Pass:                # the harness's run_* helpers silence stdout through _Quiet
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False
    orig_quiet = M._Quiet
    M._Quiet = _Pass
    try:
        with Capture() as c:
            it1 = M.run_cluster(net, "track_state_estimates", 1.0, 2.0)
        out["cluster_tse"] = parse(c.buf.getvalue())
        with Capture() as c:
            it2 = M.run_extrapolate(it1)
        out["extrapolate"] = parse(c.buf.getvalue())
        rem = M.simulate_extraction(it2)
        with Capture() as c:
            M.run_update(rem)
        out["update"] = parse(c.buf.getvalue())
    finally:
        M._Quiet = orig_quiet
    path = os.path.join(HERE, "diag_vol7.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, {k: v for k, v in out.items() if k != "truth"})


if __name__ == "__main__":
    main()
