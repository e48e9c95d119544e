"""Per-kernel averages of rocprofv3 --pmc passes (tools/pmc_kernels.sh output directories).

    python tools/pmc_summary.py gpurun_out/<name> [--min-ms 1.0]

Dispatches are grouped by kernel name and rounded duration; counters are averaged per dispatch.
Derived: clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; per-wave-cycle fractions of SQ_WAIT_ANY
(parked at s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY; MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CUs * 4 SIMDs) (MI355X_MICROARCH.md).
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    name = name.replace("void trpo::(anonymous namespace)::", "").replace("trpo::(anonymous namespace)::", "")
    return re.sub(r"\(trpo::.*", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-ms", type=float, default=1.0)
    args = ap.parse_args()
    data = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = {}
    for f in glob.glob(os.path.join(args.dir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if ms < args.min_ms:
                continue
            key = (short(r["Kernel_Name"]), round(ms, 0))
            data[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur.setdefault(key, []).append(ms)
    for key in sorted(data, key=lambda k: -k[1]):
        c = {k: sum(v) / len(v) for k, v in data[key].items()}
        ms = sum(dur[key]) / len(dur[key])
        line = [f"{key[0][:60]:60s} {ms:7.2f} ms"]
        if "GRBM_GUI_ACTIVE" in c:
            line.append(f"clk {c['GRBM_GUI_ACTIVE'] / 8 / (ms * 1e-3) / 1e9:.2f}GHz")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in c:
                    line.append(f"{k[3:]} {c[k] / wc:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            line.append(f"mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU",
                  "SQ_INSTS_VALU_FP64", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVES",
                  "SQ_VALU_MFMA_COEXEC_CYCLES"):
            if k in c:
                line.append(f"{k[3:]} {c[k]:.3g}")
        print("  ".join(line))


if __name__ == "__main__":
    main()
