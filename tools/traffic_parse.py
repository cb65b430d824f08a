"""Reduce the FETCH_SIZE / WRITE_SIZE passes of tools/prof_r01.sh to
per-dispatch HBM bytes of the last k_mpc_step dispatch and of the calibration
copy, and write profiles/traffic_<round>.json (read by bench.py)."""
import collections
import csv
import json
import sys
from pathlib import Path

outdir, B, tag = Path(sys.argv[1]), int(sys.argv[2]), sys.argv[3]


def per_dispatch(path, counter):
    d = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        d[k] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    return d, names


def pick(d, names, key):
    ks = [k for k in sorted(d) if key(names[k])]
    return d[ks[-1]] if ks else None


fetch, fn = per_dispatch(next(outdir.rglob("fetch*counter_collection.csv")), "FETCH_SIZE")
write, wn = per_dispatch(next(outdir.rglob("write*counter_collection.csv")), "WRITE_SIZE")
is_step = lambda n: "k_mpc_step" in n                                     # noqa: E731
is_copy = lambda n: "copy" in n.lower() or "elementwise" in n.lower()     # noqa: E731
KB = 1024.0                                                              # rocprofv3 reports kilobytes
f_step, w_step = pick(fetch, fn, is_step) * KB, pick(write, wn, is_step) * KB
f_cal, w_cal = pick(fetch, fn, is_copy), pick(write, wn, is_copy)
cal_bytes = 512.0 * 2 ** 20
res = {
    "round": tag, "B": B, "N": 20, "mode": 2,
    "kernel": "k_mpc_step",
    "fetch_bytes_per_launch": f_step,
    "write_bytes_per_launch": w_step,
    # the guide's prescribed correction: FETCH_SIZE x2 (it tallies 128-B requests at 64 B)
    "hbm_bytes_per_launch": 2 * f_step + w_step,
    # state in/out + outputs (1816 B) + warm-start workspace in/out (336 B), as flops.hbm_bytes_per_step
    "algorithmic_bytes_per_launch": B * (8 * (2 + 6 * 20 + 2 * 20 + 20 + 2 * 21 + 2) + 8 + 2 * 4 * 2 * 21),
    "calibration": {"copy_bytes_each_way": cal_bytes,
                    "fetch_reported": None if f_cal is None else f_cal * KB,
                    "write_reported": None if w_cal is None else w_cal * KB},
    "note": "FETCH_SIZE/WRITE_SIZE from separate --pmc passes (MI355X_MICROARCH.md HBM section), kilobytes "
            "x1024; hbm_bytes_per_launch = 2*FETCH + WRITE (the guide's x2 FETCH correction, confirmed by "
            "the calibration copy in the same run; for the step kernel's 8 B/lane loads it is an upper "
            "estimate).",
}
(outdir / f"traffic_{tag}.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
