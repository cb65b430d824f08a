"""Static instruction mix per diagnostic phase of one kernel, from the -S output
of a -DNTM_STAMPS build: each NTM_ACC(i, t) is an s_memtime followed by a
read-add-write of ntm_lds_stamps[i]; the code between two s_memtime is charged
to the stamp the second one updates.  Static counts (loops counted once), so a
guide to what a phase is made of, not a timing.

    python tools/isa_phases.py /tmp/diag20.s [kernel-substring]
"""
import re
import sys
from collections import Counter, defaultdict

NAMES = ("ST_LIFT ST_COST ST_SCALE ST_CAND ST_REGRAM ST_GI ST_POLISH ST_ROLL ST_GI_FACT ST_GI_CHECK "
         "ST_GI_DIR ST_GI_ADD ST_GI_DROP CN_CHECK CN_CAND CN_HIT ST_P_CLASS ST_P_GRAM ST_P_CHOL ST_P_SCHUR "
         "ST_P_BWD ST_P_KKT CN_REPAIR CN_GIRUN ST_S_E ST_S_Y ST_S_K ST_S_CHOL ST_S_SOLVE CN_TRY_EARLY "
         "CN_FAIL_EARLY CN_FAIL_LATE CN_FAIL_IT1 CN_FAIL_IT2 CN_GI_IT1 CN_GI_IT2 CN_GI_LATE CN_TRY_IT1 "
         "CN_TRY_IT2 CN_WARM_TRY CN_WARM_OK CN_WARM_DEP CN_WARM_NEG CN_WARM_FULL CN_ALT_TRY CN_ALT_HIT "
         "ST_K_Y ST_K_CHK ST_K_GRAD ST_K_MU ST_K_SUB ST_C_A ST_C_B ST_C_Y ST_C_SQ ST_SC_COL ST_SC_ROW "
         "ST_SC_END ST_L_COEF ST_L_LOOP").split()
F64 = re.compile(r"^v_(fma|mul|add|fmac|max|min|rcp|rsq|sqrt|div_fmas|div_fixup|div_scale|ldexp|frexp|fract|trig|cmp\w*)_f64")


def classify(op):
    if op.startswith("v_"):
        if F64.match(op):
            return "f64"
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            return "lane"
        if "dpp" in op or op.startswith(("v_mov_b32_dpp", "v_permlane")):
            return "dpp"
        if op.startswith(("v_cndmask", "v_cmp")):
            return "mask"
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_mpc_step"
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("_Z") and pat in ln.split(":")[0] and ":" in ln)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = [ln.strip() for ln in lines[start:end]]
    seg = Counter()
    total = defaultdict(Counter)
    i = 0
    while i < len(body):
        ln = body[i]
        op = ln.split()[0] if ln and not ln.startswith((";", ".")) else ""
        if op == "s_memtime":
            # the stamp this s_memtime closes: next ds_read_b64 off the stamps base
            idx = None
            for k in range(i + 1, min(i + 14, len(body))):
                m = re.match(r"ds_read_b64 v\[\d+:\d+\], v\d+(?: offset:(\d+))?$", body[k])
                if m:
                    off = int(m.group(1) or 0)
                    if off % 8 == 0 and off // 8 < len(NAMES):
                        idx = off // 8
                    break
            name = NAMES[idx] if idx is not None else "?"
            total[name].update(seg)
            seg = Counter()
        elif op:
            seg[classify(op)] += 1
        i += 1
    total["(tail)"].update(seg)
    keys = ("f64", "valu", "mask", "dpp", "lane", "salu", "lds", "scratch", "vmem", "other")
    print(f"{'phase':12s} " + " ".join(f"{k:>7s}" for k in keys) + "   total")
    for name, c in sorted(total.items(), key=lambda kv: -sum(kv[1].values())):
        print(f"{name:12s} " + " ".join(f"{c[k]:7d}" for k in keys) + f"   {sum(c.values()):5d}")


if __name__ == "__main__":
    main()
