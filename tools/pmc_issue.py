"""Issue-stall attribution of a kernel from the scripts/pmc_issue.txt passes (two rocprofv3 --pmc runs):
mean per dispatch of each SQ counter, and the shares of the wave cycles.  Development tool.

    python tools/pmc_issue.py gpurun_out/<tag>/<session> [kernel-substring ...]

SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt / barriers) + SQ_WAIT_INST_ANY (ready but the instruction
cannot issue: a dependency or a busy pipe) + SQ_ACTIVE_INST_ANY (issuing), disjoint (MI355X_MICROARCH.md
"rocprofv3 PMC slots"); SQ_WAIT_INST_LDS is the LDS part of WAIT_INST_ANY.  ACTIVE_INST_VALU / _SCA / _LDS
split the issuing cycles by unit.  All in the counters' own (quad-cycle) units, summed over the chip.
"""
import collections
import csv
import glob
import os
import sys


def load(session):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(session, "pmc*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main():
    session, subs = sys.argv[1], sys.argv[2:] or ["render_bwd", "render_fwd"]
    k = load(session)
    for name, c in sorted(k.items()):
        if not any(s in name for s in subs):
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"## {name[:90]}")
        for key in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM",
                    "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if key in c:
                print(f"  {key:22s} {c[key]:12.4g}")
        for key in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                    "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS"):
            if key in c:
                print(f"  {key:22s} {c[key]:12.4g}  {c[key] / wc:6.3f} of wave cycles")


if __name__ == "__main__":
    main()
