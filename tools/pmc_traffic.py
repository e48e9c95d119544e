"""Per-launch HBM traffic of the bench's hot kernels from rocprofv3 PMC passes (tools/prof.sh).

    python tools/pmc_traffic.py gpurun_out/<name> profiles/<round>/traffic.json --config c4 --rows 8000000

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md (HBM/rocprofv3):
on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide (16 B/lane) streaming reads, so
read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for streaming stores.  The hot
kernels' operand loads are 16 B/lane streams; their epilogue loads are 4 B/lane row
segments (whole 128-B lines per 32 lanes), for which the same factor held: the
R-backward launches read 2 x FETCH = 42.3 GB against 41.9 GB of algorithmic bytes.

A bench tag is matched to dispatches by kernel name plus its position in the fixed
launch order of one FVP (e.g. the two kRBwd row GEMMs of an FVP are l=2 then l=1).
"""
import argparse
import csv
import json
import os
import statistics
import sys

# tag -> (kernel-name substring, period, phase): the phase-th of every `period` dispatches
# (kernel template arguments as rocprofv3 prints them; the last rowgemm3/wgrad3 argument is the
# plane count: 2 = the default f16 split)
SPECS = {
    "fvp_rfwd_l0": ("rowgemm_pl_kernel<1, 1>", 1, 0),                       # X planes, kRHidden (plane.hip)
    "fvp_rfwd_l1": ("rowgemm3_kernel<4, 2, 2, 4, 11, 2, 1, 2, 32>", 1, 0),  # kRZ into the tail (BK 32)
    "fvp_rfwd01": ("rfwd01_kernel<8>", 1, 0),                               # layers 0 + 1 R-forward (rfwd.hip)
    "fvp_rbwdwg_l1": ("rbwd0_kernel<2>", 1, 0),                             # R-backward + X^T RD_0 (rbwd0.hip)
    "fvp_tail_l2": ("fvp_tail_kernel", 1, 0),
    # C2 / C3: the one-launch FVP (fused16.hip <FW, LB, TI0, OTA, MODE, NH> with MODE 0, the only zero argument;
    # every substring must be in the name)
    "fvp_fused": (("fvp_fused16_kernel<", ", 0, "), 1, 0),
}
# tags whose kernel is shared with a 1-segment policy-gradient launch: keep the long ones
LONGEST = {
    "fvp_wgrad_l1": "wgrad3_kernel<4, 2, 2, 4, 2, 1, 2>",
}


def load(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    rows.sort()
    return rows


def pick(rows, sub, period=None, phase=None, longest=False):
    subs = sub if isinstance(sub, tuple) else (sub,)
    sel = [r for r in rows if all(x in r[1] for x in subs)]
    if longest and sel:
        # the FVP launches are the majority: keep those near the median duration (a single dispatch
        # slowed down under the counters must not become the reference)
        dmed = statistics.median(r[3] for r in sel)
        sel = [r for r in sel if r[3] > 0.75 * dmed]
    elif period:
        sel = [r for i, r in enumerate(sel) if i % period == phase]
    return sel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--rows", type=int, default=8_000_000)
    a = ap.parse_args()
    fetch = load(os.path.join(a.pmc_dir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(a.pmc_dir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import source_build_id
    res = {"config": a.config, "rows": a.rows, "source": a.pmc_dir, "build": source_build_id(),
           "method": "read = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane streams), write = WRITE_SIZE; "
                     "KiB -> bytes x 1024; mean over the matched launches", "tags": {}}
    todo = [(t, s, p, ph, False) for t, (s, p, ph) in SPECS.items()] + \
           [(t, s, None, None, True) for t, s in LONGEST.items()]
    for tag, sub, period, phase, longest in todo:
        f = pick(fetch, sub, period, phase, longest)
        w = pick(write, sub, period, phase, longest)
        if not f or not w:
            continue
        rd = 2 * 1024 * statistics.mean(r[2] for r in f)
        wr = 1024 * statistics.mean(r[2] for r in w)
        res["tags"][tag] = {"kernel": "".join(sub) if isinstance(sub, tuple) else sub, "launches": len(f), "read_bytes": rd, "write_bytes": wr,
                            "traffic_bytes": rd + wr, "pmc_run_ms": statistics.mean(r[3] for r in f)}
    res["fvp_total_bytes"] = sum(v["traffic_bytes"] for v in res["tags"].values())
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    for t, v in res["tags"].items():
        print(f"{t:14s} {v['launches']:4d}  read {v['read_bytes'] / 1e9:7.2f} GB  write {v['write_bytes'] / 1e9:6.2f} GB"
              f"  {v['pmc_run_ms']:7.2f} ms")
    print(f"FVP total {res['fvp_total_bytes'] / 1e9:.1f} GB")


if __name__ == "__main__":
    main()
