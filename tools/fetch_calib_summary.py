"""Turn the tools/gpu_fetch_calib.sh passes into profiles/fetch_calibration.json (dev tool).

usage: python tools/fetch_calib_summary.py DIR   (DIR holds pmc_fetch.csv, pmc_write.csv, pmc_req.csv
or the rocprofv3 output dirs pmc_fetch/ pmc_write/ pmc_req/)
factor = known bytes / (counter kB * 1024) per access shape of tools/fetch_calib.hip.
"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READ = WRITE = 1 << 30


def load(name):
    f = os.path.join(d, name + ".csv")
    if not os.path.exists(f):
        f = glob.glob(os.path.join(d, name, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0], r["Counter_Name"])
            agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"])
    return agg


fetch, write, req = load("pmc_fetch"), load("pmc_write"), load("pmc_req")
out = {"source": "tools/fetch_calib.hip under rocprofv3 --pmc (tools/gpu_fetch_calib.sh), one pass per counter",
       "bytes_read_per_kernel": READ, "bytes_written_per_write_kernel": WRITE, "shapes": {}}
for (disp, kern, ctr), v in sorted(fetch.items()):
    if kern.startswith("read_"):
        rq = req.get((disp, kern, "TCC_EA0_RDREQ_sum"))
        out["shapes"][kern] = {"FETCH_SIZE_kB": v, "fetch_factor": READ / (v * 1024),
                               "TCC_EA0_RDREQ": rq, "bytes_per_rdreq": READ / rq if rq else None}
wf = [READ / (v * 1024) for (disp, kern, ctr), v in write.items() if kern == "write_dword"]
out["write_dword_factor"] = sum(wf) / len(wf)
ff = [s["fetch_factor"] for s in out["shapes"].values()]
out["fetch_factor"] = round(sum(ff) / len(ff), 4)
out["note"] = ("FETCH_SIZE reports half the bytes for 4 B/lane dword, 4 B/lane SoA (field*n_envs+env) and "
               "16 B/lane dwordx4 reads alike (128-B EA read requests tallied at 64 B); WRITE_SIZE is exact "
               "for 4 B/lane dword stores.  pmc_summary.py applies fetch_factor / write_dword_factor.")
with open(os.path.join(REPO, "profiles", "fetch_calibration.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
