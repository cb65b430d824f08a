"""Reduce the SQ passes of tools/prof_pmc.sh (pmc1 + pmc2 counter CSVs) to the
last k_mpc_step dispatch and write profiles/sq_<round>.json-style output: the
wave-cycle split (issuing / parked on s_waitcnt / issue-stalled) and the VALU
instruction mix.  SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_INST_* count
quad-cycles (MI355X_MICROARCH.md, PMC units table); ratios between them are
unit-free."""
import collections
import csv
import json
import sys
from pathlib import Path

outdir, tag = Path(sys.argv[1]), sys.argv[2]
# resident waves per SIMD of the measured build (N=20: 3 since the far workspace, round 3; 2 before)
wps = int(sys.argv[3]) if len(sys.argv) > 3 else 4   # N = 20 slim layout: 4 waves per SIMD (round 5)


def last_step(path):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "k_mpc_step" not in r["Kernel_Name"]:
            continue
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return d[max(d)] if d else {}


c = {}
for f in sorted(outdir.rglob("pmc*_counter_collection.csv")):
    c.update(last_step(f))
waves = c.get("SQ_WAVES", 0.0)
wc = c.get("SQ_WAVE_CYCLES", 0.0)
valu = c.get("SQ_INSTS_VALU", 0.0)
f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                   "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"))
res = {
    "round": tag,
    "kernel": "k_mpc_step<64,20>",
    "counters_per_launch": dict(sorted(c.items())),
    "per_wave": {k: v / waves for k, v in sorted(c.items()) if waves and k != "SQ_WAVES"},
    "derived": {
        "valu_issue_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc if wc else None,
        "parked_waitcnt_frac_of_wave_cycles": c.get("SQ_WAIT_ANY", 0.0) / wc if wc else None,
        "issue_stall_frac_of_wave_cycles": c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else None,
        "fp64_arith_frac_of_valu_insts": f64 / valu if valu else None,
        "waves_per_simd": wps,
        "simd_valu_busy_estimate": wps * c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc if wc else None,
    },
    "note": "separate --pmc passes (8 SQ counters each) over one bench step at B=1e5, N=20; the "
            "SIMD VALU busy estimate is waves/SIMD x the per-wave VALU-issue fraction.",
}
(outdir / f"sq_{tag}.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res["derived"], indent=1))
