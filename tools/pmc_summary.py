#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel and write profiles/traffic.json.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the read-side factor 2 is the guide's
calibration for 16-B-per-lane streams; write side exact).

    python tools/pmc_summary.py gpurun_out/<tag>_pmc [--batch 64 --size 256 --out profiles/traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

LAYER_OF = [  # kernel-name pattern -> bench layer name (order matters: first match)
    (r"conv1_colour", "conv1"), (r"dconv8_colour", "dconv8"), (r"dconv8_x3", "dconv8"), (r"dconv8_strip", "dconv8"),
    (r"conv12_kernel", "conv2"), (r"conv_ws2_kernel<32, 64", "conv2"), (r"conv_ws2_kernel<64, 32", "conv8"),
    (r"<32, 64, 5, 2, false", "conv2"), (r"<64, 32, 5, 2, false", "conv8"),
    (r"<32, 64, 5, 2, true", "dconv1"), (r"<64, 64, 5, 2, true", "dconv7"),
    (r"dconv8_gather", "dconv8"), (r"conv_ws_kernel<64, 64, 8, 8, false, true", "dconv7"),
    (r"conv_ws_kernel<64, 64, 8, 8, true, false", "k3_resid"), (r"conv_ws_kernel<64, 64, 8, 8, false, false", "k3"),
    (r"<64, 64, 3, 1, false.*true>", "k3_resid"), (r"<64, 64, 3, 1, false.*false>", "k3"),
    (r"latent_hist", "hist"), (r"hist_entropy", "entropy"), (r"conv_k3pair_kernel", "k3_pair"),
    (r"dconv1_all_kernel", "dconv1"),
    (r"colour_split", "colour"), (r"fp32_chain", "fp32_chain"), (r"dconv1_ws_kernel", "dconv1"),
]


def layer_of(name):
    for pat, lay in LAYER_OF:
        if re.search(pat, name):
            return lay
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))  # layer -> counter -> per-dispatch values
    for f in glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))  # (dispatch, kernel) -> counter -> sum
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row.get("Dispatch_Id"), row.get("Kernel_Name"))
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
        for (disp, kname), cs in per.items():
            lay = layer_of(kname or "")
            if lay:
                for c, v in cs.items():
                    vals[lay][c].append(v)
    summary = {}
    for lay, cs in sorted(vals.items()):
        # drop the warm-up dispatches' variance by taking the median per counter
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        d = {c: med[c] for c in sorted(med)}
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            d["hbm_bytes_per_launch"] = int((2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024)
        if "SQ_LDS_BANK_CONFLICT" in med and "SQ_LDS_IDX_ACTIVE" in med and med["SQ_LDS_IDX_ACTIVE"] > 0:
            d["lds_bank_conflict_frac"] = med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"]
        wc = med.get("SQ_WAVE_CYCLES", 0)
        if wc > 0:  # disjoint wave-state buckets (guide: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
            for c, k in (("SQ_WAIT_ANY", "wave_waitcnt_barrier_frac"), ("SQ_WAIT_INST_ANY", "wave_issue_stall_frac"),
                         ("SQ_ACTIVE_INST_ANY", "wave_issuing_frac")):
                if c in med:
                    d[k] = med[c] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and med.get("GRBM_GUI_ACTIVE", 0) > 0:
            # per-SIMD MFMA busy fraction: counter summed over 256 CUs x 4 SIMDs, GRBM in GPU cycles
            d["mfma_busy_frac"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * med["GRBM_GUI_ACTIVE"] / 8)
        summary[lay] = d
    # the k3 kernels serve conv3/dconv5 and conv4/dconv6
    # (the fused residual pair k3_pair is timed as conv4 / dconv6 and replaces both)
    for a, b in (("k3", ("conv3", "dconv5")), ("k3_resid", ("conv4", "dconv6")), ("k3_pair", ("conv4", "dconv6"))):
        if a in summary:
            for x in b:
                summary[x] = summary[a]
    out = {"batch": args.batch, "size": args.size, "source": os.path.relpath(args.pmc_dir).replace("gpurun_out", "profiles"),
           "method": "(2*FETCH_SIZE + WRITE_SIZE)*1024 per dispatch, median over dispatches",
           "layers": summary}
    json.dump(out, sys.stdout, indent=1)
    print()
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
