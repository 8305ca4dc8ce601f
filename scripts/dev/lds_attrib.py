"""Per-section LDS counters of the step kernel from scripts/dev/lds_attrib.sh
output (developer tool): counter(stop k) - counter(previous stop), per wave.

    python scripts/dev/lds_attrib.py gpurun_out/ldsattr [ThormangWalk Gogoro]
"""
import json
import os
import sys

ORDER = [("0", "load"), ("16", "1a schedule fwd"), ("1", "1b all groups"), ("17", "2a all groups"),
         ("18", "2b schedule bwd"), ("2", "root solve"), ("3", "pass 3"), ("4", "contact rows"),
         ("5", "delassus"), ("6", "pgs setup"), ("7", "pgs + apply"), ("8", "integrate"),
         ("full", "rest of the substeps + store")]
CTR = ["SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES"]


def load(root, task, k):
    d = json.load(open(os.path.join(root, f"{task}_{k}.json")))
    e = d["step_par_kernel"]["avg"]
    w = e["SQ_WAVES"]
    return {c: e.get(c, 0.0) / w for c in CTR}


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ldsattr"
    tasks = sys.argv[2:] or ["ThormangWalk", "Gogoro"]
    for task in tasks:
        if not os.path.exists(os.path.join(root, f"{task}_full.json")):
            continue
        print(f"# {task}: step_par_kernel per wave, first substep by section (stop-point builds)")
        print(f"{'section':30s} {'LDS instr':>10s} {'LDS active':>11s} {'conflict':>9s} {'confl/act':>9s} "
              f"{'VALU instr':>10s}")
        prev = {c: 0.0 for c in CTR}
        tot = load(root, task, "full")
        for k, name in ORDER:
            cur = load(root, task, k)
            d = {c: cur[c] - prev[c] for c in CTR}
            fr = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"] if d["SQ_LDS_IDX_ACTIVE"] > 0 else 0.0
            print(f"{name:30s} {d['SQ_INSTS_LDS']:10.0f} {d['SQ_LDS_IDX_ACTIVE']:11.0f} "
                  f"{d['SQ_LDS_BANK_CONFLICT']:9.0f} {fr:9.3f} {d['SQ_INSTS_VALU']:10.0f}")
            prev = cur
        fr = tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_LDS_IDX_ACTIVE"]
        print(f"{'whole kernel':30s} {tot['SQ_INSTS_LDS']:10.0f} {tot['SQ_LDS_IDX_ACTIVE']:11.0f} "
              f"{tot['SQ_LDS_BANK_CONFLICT']:9.0f} {fr:9.3f} {tot['SQ_INSTS_VALU']:10.0f}\n")


if __name__ == "__main__":
    main()
