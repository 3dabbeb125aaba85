"""Summarise tools/gpu_stalls.sh passes into profiles/ROUND_stalls_summary.json (dev tool).

usage: python tools/stalls_summary.py gpurun_out/TAG ROUND
Per-dispatch medians of the two metric step kernels; SQ_* cycle counters are in quad-cycles,
so the fractions of SQ_WAVE_CYCLES are unit-free.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

src, rnd = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {}
WORK = (("ant", "pbg_models::Ant", False), ("humanoid", "pbg_models::Humanoid", False), ("ant_f64", "pbg_models::Ant", True),
        ("humanoid_f64", "pbg_models::Humanoid", True))
for w, key, f64 in WORK:
    if not glob.glob(os.path.join(src, w, "pmc_wait", "**", "*counter_collection.csv"), recursive=True):
        continue
    r = {}
    for d in ("pmc_wait", "pmc_lds"):
        f = glob.glob(os.path.join(src, w, d, "**", "*counter_collection.csv"), recursive=True)[0]
        shutil.copy(f, os.path.join(REPO, "profiles", f"{rnd}_{d}_{w}.csv"))
        per = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "step_kernel" in name and key in name and (("F64<" in name) == f64):
                    per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                    per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        r.update({k: statistics.median(v.values()) for k, v in per.items()})
    wc = r["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        r["frac_" + k[3:].lower()] = r[k] / wc
    r["lds_bank_conflict_per_lds_active"] = r["SQ_LDS_BANK_CONFLICT"] / max(r["SQ_LDS_IDX_ACTIVE"], 1)
    res[w] = r
res["source"] = ("tools/gpu_stalls.sh (python bench.py --steps 20 --warmup 2, one --pmc pass of 8 SQ counters "
                 "each); per-dispatch medians of the step kernel")
with open(os.path.join(REPO, "profiles", f"{rnd}_stalls_summary.json"), "w") as f:
    json.dump(res, f, indent=1)
for w in (w for w, _, _ in WORK if w in res):
    print(w, {k: round(v, 3) for k, v in res[w].items() if k.startswith(("frac", "lds"))})
