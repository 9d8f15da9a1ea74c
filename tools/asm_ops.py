"""Static instruction counts per node op of the fused node kernel, from an assembly listing
built with -DGTF_ASM_MARK=1 (every op preceded by a '; GTF_OP_MARK G=.. OP=..' line):
instructions between one marker and the next, attributed to the op of the first. The
compiler may move code across the markers (they are only asm comments with no operands),
so the split is approximate; loops count once.
    hipcc ... -DGTF_ASM_MARK=1 --cuda-device-only -S -o mark.s gtf_pass.hip
    python tools/asm_ops.py mark.s <kernel substring>"""
import collections
import re
import sys

OPS = {1: "ranks", 2: "priors_tse", 3: "priors_uts", 4: "reweight", 5: "degree", 6: "prune", 7: "mw_tse",
       8: "mw_uts", 9: "cluster_tse", 10: "cluster_uts", 11: "fresh", 12: "flush", 99: "store", 100: "end"}


def main():
    f, pat = sys.argv[1], sys.argv[2]
    L = open(f).read().split("\n")
    start = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + pat + r"\S*:", l))
    end = start + 1
    while not L[end].startswith(".Lfunc_end"):
        end += 1
    cur = ("pre", 0)
    cnt = collections.defaultdict(collections.Counter)
    for l in L[start:end]:
        m = re.search(r"GTF_OP_MARK G=(\d+) OP=(\d+)", l)
        if m:
            cur = (int(m.group(1)), OPS.get(int(m.group(2)), m.group(2)))
            continue
        t = l.strip()
        if not l.startswith("\t") or not t or t.startswith((".", ";")):
            continue
        ins = t.split()[0]
        k = "valu" if ins.startswith("v_") else "salu" if ins.startswith("s_") else "lds" if ins.startswith("ds_") \
            else "vmem" if ins.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
        cnt[cur][k] += 1
        if ins.startswith("v_div_fixup"):
            cnt[cur]["div"] += 1
        if "cndmask" in ins:
            cnt[cur]["cndmask"] += 1
        if ins.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane")):
            cnt[cur]["mov"] += 1
        if ins.startswith("v_cmp"):
            cnt[cur]["cmp"] += 1
        if "_f64" in ins:
            cnt[cur]["f64"] += 1
    for G in (64, 32, 16, 8, 4, 2):
        rows = [(k, v) for k, v in cnt.items() if k[0] == G]
        if not rows:
            continue
        tot = sum(v["valu"] for _, v in rows)
        print("G=%d  VALU %d" % (G, tot))
        for k, v in rows:
            print("   %-12s valu %5d (f64 %4d div %2d cndmask %4d mov %4d cmp %4d) salu %5d lds %4d vmem %4d" % (
                k[1], v["valu"], v["f64"], v["div"], v["cndmask"], v["mov"], v["cmp"], v["salu"], v["lds"], v["vmem"]))


if __name__ == "__main__":
    main()
