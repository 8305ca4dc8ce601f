"""LDS bank-conflict model of the step kernel's main access patterns (developer
tool): for an env stride ES (floats) and group stride GF, the extra LDS cycles
per wave-instruction of the tree passes' and the all-groups passes' reads,
with the lane groups / bank rules of /opt/skills/guides/MI355X_MICROARCH.md
§LDS (ds_read_b32: 2 x 32 lanes, 32 banks; ds_read_b64: 2 x 32, 64 banks;
ds_read_b128: 4 x 16 lane groups {0-3,12-15,20-27}, ..., 64 banks).

    python scripts/dev/lds_bank_model.py [model] [max_pad]
"""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def parse(name):
    txt = open(os.path.join(REPO, "thormang_isaacgym_amd", "csrc", "generated", f"Model_{name}.inc")).read()
    g = lambda k: int(re.search(rf"\b{k} = (\d+)", txt).group(1))
    sched = eval(re.search(r"sched\[\d+\]\[\d+\] = (\{.*?\}\});", txt).group(1).replace("{", "[").replace("}", "]"))
    parent = eval(re.search(r"int parent\[\d+\] = (\{.*?\});", txt).group(1).replace("{", "[").replace("}", "]"))
    return dict(NG=g("NG"), LPE=g("LPE"), SL=g("SL"), sched=sched, parent=parent)


def extra_cycles(addrs, width):
    """addrs[lane] = float address or None (inactive); extra cycles over the ideal."""
    if width == 16:
        groups, nb = B128_GROUPS, 64
    else:
        groups, nb = [list(range(0, 32)), list(range(32, 64))], (64 if width == 8 else 32)
    extra = 0
    for grp in groups:
        banks = {}
        for l in grp:
            a = addrs[l]
            if a is None:
                continue
            for k in range(width // 4):
                b = (a + k) % nb
                banks.setdefault(b, set()).add(a + k)
        worst = max((len(v) for v in banks.values()), default=1)
        extra += worst - 1
    return extra


def model_cost(m, ES, GF=60):
    LPE, SL = m["LPE"], m["SL"]
    epw = 64 // LPE
    tot = 0
    # tree steps: each lane reads its slot's group (own fields) and its parent (1a)
    for row in m["sched"]:
        for field, width, who in ((0, 16, "par"), (4, 16, "par"), (8, 16, "par"), (12, 8, "par"),
                                  (20, 16, "own"), (26, 8, "own"), (35, 8, "own"), (44, 16, "own"), (50, 8, "own"),
                                  (41, 4, "own"), (42, 4, "own"), (18, 4, "own"), (19, 4, "own")):
            addrs = []
            for lane in range(64):
                e, sub = divmod(lane, LPE)
                g = row[sub % SL]
                if g <= 0:
                    addrs.append(None)
                    continue
                gg = m["parent"][g] if who == "par" else g
                addrs.append(e * ES + gg * GF + field)
            tot += extra_cycles(addrs, width)
    # all-groups rounds (1b, 2a, integrate): lane sub handles group sub + LPE r
    for r in range((m["NG"] + LPE - 1) // LPE):
        for field, width in ((0, 16), (4, 16), (8, 16), (12, 8), (18, 4), (19, 4), (20, 16), (24, 16), (44, 16)):
            addrs = []
            for lane in range(64):
                e, sub = divmod(lane, LPE)
                g = sub + LPE * r
                addrs.append(e * ES + g * GF + field if g < m["NG"] else None)
            tot += extra_cycles(addrs, width)
    return tot


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "thormang"
    maxpad = int(sys.argv[2]) if len(sys.argv) > 2 else 76
    m = parse(name)
    ES0 = int(sys.argv[3]) if len(sys.argv) > 3 else None
    if ES0 is None:
        raise SystemExit("give the current env stride ES (floats) as the third argument")
    base = model_cost(m, ES0)
    print(f"{name}: ES {ES0} (mod 64 = {ES0 % 64}) extra cycles {base}")
    for pad in range(0, maxpad + 1, 4):
        c = model_cost(m, ES0 + pad)
        print(f"  pad {pad:3d}  ES {ES0 + pad}  mod64 {(ES0 + pad) % 64:2d}  extra {c:5d}  ({c / max(base, 1):.2f}x)")
