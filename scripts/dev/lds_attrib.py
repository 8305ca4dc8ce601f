"""Per-section SQ counters of the step kernel from scripts/dev/lds_attrib.sh
output (developer tool): counter(stop k) - counter(previous stop), per wave,
every counter the passes collected (LDS conflict fraction when both LDS
counters are there).

    python scripts/dev/lds_attrib.py gpurun_out/ldsattr [ThormangWalk Gogoro]
"""
import json
import os
import sys

ORDER = [("0", "load"), ("16", "1a schedule fwd"), ("1", "1b all groups"), ("17", "2a all groups"),
         ("18", "2b schedule bwd"), ("2", "root solve"), ("3", "pass 3"), ("4", "contact rows"),
         ("5", "delassus"), ("6", "pgs"), ("7", "impulse application"), ("8", "integrate"),
         ("full", "rest of the substeps + store")]
SHORT = {"SQ_INSTS_LDS": "LDS instr", "SQ_LDS_IDX_ACTIVE": "LDS active", "SQ_LDS_BANK_CONFLICT": "conflict",
         "SQ_INSTS_VALU": "VALU instr", "SQ_WAVE_CYCLES": "wave cyc", "SQ_WAIT_ANY": "waitcnt",
         "SQ_WAIT_INST_ANY": "issue stall", "SQ_ACTIVE_INST_VALU": "VALU act", "SQ_ACTIVE_INST_LDS": "LDS act",
         "SQ_ACTIVE_INST_ANY": "any act", "SQ_WAIT_INST_LDS": "LDS q stall"}


def load(root, task, k):
    d = json.load(open(os.path.join(root, f"{task}_{k}.json")))
    e = d["step_par_kernel"]["avg"]
    w = e["SQ_WAVES"]
    return {c: v / w for c, v in e.items() if c != "SQ_WAVES"}


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ldsattr"
    tasks = sys.argv[2:] or ["ThormangWalk", "Gogoro"]
    for task in tasks:
        if not os.path.exists(os.path.join(root, f"{task}_full.json")):
            continue
        tot = load(root, task, "full")
        ctr = sorted(tot)
        lds = "SQ_LDS_BANK_CONFLICT" in tot and "SQ_LDS_IDX_ACTIVE" in tot
        print(f"# {task}: step_par_kernel per wave, first substep by section (stop-point builds)")
        print(f"{'section':30s} " + " ".join(f"{SHORT.get(c, c):>11s}" for c in ctr) + (" confl/act" if lds else ""))
        prev = {c: 0.0 for c in ctr}
        rows = [(k, n, load(root, task, k)) for k, n in ORDER] + [(None, "whole kernel", None)]
        for k, name, cur in rows:
            d = tot if cur is None else {c: cur.get(c, 0.0) - prev[c] for c in ctr}
            line = f"{name:30s} " + " ".join(f"{d[c]:11.0f}" for c in ctr)
            if lds:
                fr = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"] if d["SQ_LDS_IDX_ACTIVE"] > 0 else 0.0
                line += f" {fr:9.3f}"
            print(line)
            if cur is not None:
                prev = cur
        print()


if __name__ == "__main__":
    main()
