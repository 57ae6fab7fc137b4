"""Per-launch PMC counters of the frame-build kernels from rocprofv3 --pmc CSV directories
(one per counter group): python3 pmc_table.py OUT_DIR [OUT_JSON].  Each dispatch row repeats
the whole launch's value (8 rows per dispatch, one per XCD dimension entry), so the mean over
rows is the per-launch value."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_collect import setup_dispatches  # noqa: E402

out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "pmc_*", "**", "*counter_collection.csv"), recursive=True):
    cfg = os.path.relpath(f, sys.argv[1]).split(os.sep)[0][4:]
    for g in ("_WRITE_SIZE", "_FETCH_SIZE", "_G1", "_G2", "_G3"):
        cfg = cfg[: -len(g)] if cfg.endswith(g) else cfg
    rows = list(csv.DictReader(open(f)))
    want = lambda kn: kn.startswith("void pb_") and "len_" not in kn and "scan" not in kn and "fill" not in kn  # noqa
    # load-time setup dispatches (pb_ximg_body's image pages built in pbgpu_load_sequence) precede a
    # kernel's first build launch: a kernel's leading dispatches at another grid than its last
    # dispatch's are dropped (pmc_collect.setup_dispatches), every later one counts
    setup = setup_dispatches(rows, want)
    for r in rows:
        kn = r["Kernel_Name"]
        if want(kn) and r["Dispatch_Id"] not in setup:
            out[(cfg, kn.split("(")[0][5:])][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for (cfg, kn), cs in sorted(out.items()):
    d = {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())}
    if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_frac"] = round(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"], 4)
    res[f"{cfg} {kn}"] = d
    print(cfg, kn, json.dumps(d))
if len(sys.argv) > 2:
    json.dump(res, open(sys.argv[2], "w"), indent=1)
