#!/usr/bin/env python3
"""Summarise a tools/prof.sh run into profiles/<prefix>_pmc.json and
profiles/<prefix>_kernel_stats.csv.

Per kernel (base names of the untruncated rocprofv3 names, see short_name): calls and mean duration (kernel trace +
--stats), the mean FETCH_SIZE / WRITE_SIZE per dispatch from the two
separate --pmc passes (KB), and HBM bytes per dispatch and per step.

gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE reads exactly half
the bytes of a coalesced streaming read.  Checked here on known byte counts
for both widths: k_row_norms and k_chunk_sums_fast (8 B per lane) stream the
20.48 GB of fp64 rows and read 10.0e6 KB; k_screen (16 B per lane) streams
the 7.76 GB row image and reads 3.84e6 KB.  So FETCH_SIZE is doubled for the
streaming kernels (FETCH_X2); gathers and other patterns are marked
uncalibrated and taken as they are.  WRITE_SIZE is exact for streaming
stores.  Fabric-side counts include Infinity-Cache hits.

usage: tools/pmc_summary.py gpurun_out/<tag> profiles/<prefix> <rows> <iterations>
  rows: rows per GPU of the profiled run; iterations: warmup + steps.
"""
import collections
import csv
import json
import os
import sys

FETCH_X2 = {"k_screen", "k_screen32", "k_tiles_margin", "k_tiles_grad", "k_tiles_rows", "k_csr_densify",
            "k_gram_tiles", "k_gram_dma", "k_gram_dma_cov", "k_rows_quantize", "k_chunk_sums_fast", "k_chunk_sums",
            "k_row_norms", "k_rows_quantize_pf", "k_rows_quantize_q4", "k_col_partial", "k_mlr_margins", "k_mlr_grad", "k_binlog_dense", "k_binlog_csr_mult8",
            "k_binlog_csc_grad_blk", "k_summ_dense"}


def short_name(full):
    """Kernel base name from a full (untruncated) rocprofv3 name; the two
    passes of the d <= 256 KMeans screen (k_screen32<S, W, LIMBS, LIST>)
    become k_screen32_l2 / k_screen32_l3."""
    name = full.replace("(anonymous namespace)", "").split("(")[0].strip()
    if name.startswith("void "):
        name = name[5:]
    tmpl = ""
    if "<" in name:
        name, tmpl = name.split("<", 1)
    base = name.split("::")[-1].strip()
    if base == "k_screen32" and tmpl:
        args = [a.strip() for a in tmpl.rstrip(">").split(",")]
        if len(args) >= 3:
            base += "_l" + args[2]
    if base == "k_screen_cands3" and tmpl:
        # the carried sets' re-check (RC = true) apart from the candidate tier
        args = [a.strip() for a in tmpl.rstrip(">").split(",")]
        if len(args) >= 3 and args[2] == "true":
            base = "k_screen_cands3_rc"
    if base == "k_gram_dma" and tmpl:
        # the centred covariance form (MEAN 1 / 2) apart from the plain syrk
        # (MEAN 0, with or without the riding column sums): bench.py's timer
        # names
        if tmpl.split(",")[0].strip() in ("1", "2"):
            base = "k_gram_dma_cov"
    return base


def mean_counter(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(short_name(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def kernel_stats(path):
    """rocprofv3 --stats rows merged per short name (calls summed, mean
    duration weighted by calls)."""
    acc = {}
    for r in csv.DictReader(open(path)):
        n = short_name(r["Name"])
        c, t = int(r["Calls"]), float(r["TotalDurationNs"])
        a = acc.setdefault(n, {"calls": 0, "total_ns": 0.0, "pct": 0.0})
        a["calls"] += c
        a["total_ns"] += t
        a["pct"] += float(r["Percentage"])
    return {n: {"calls": a["calls"], "avg_ns": a["total_ns"] / max(a["calls"], 1),
                "pct": a["pct"]} for n, a in acc.items()}


def main(src, dst_prefix, rows, iters):
    ks = os.path.join(src, "trace", "run_kernel_stats.csv")
    stats = kernel_stats(ks)
    fetch = mean_counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = mean_counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    out = {"_rows": int(rows), "_iterations": int(iters),
           "_note": "fetch_kb_raw is rocprofv3 FETCH_SIZE per dispatch; hbm bytes use the "
                    "corrected fetch plus WRITE_SIZE"}
    for name, s in stats.items():
        f = fetch.get((name, "FETCH_SIZE"))
        w = write.get((name, "WRITE_SIZE"))
        if name in FETCH_X2 or name.rsplit("_l", 1)[0] in FETCH_X2:
            fac, cal = 2.0, "x2 (streaming read, gfx950 half count)"
        else:
            fac, cal = 1.0, "uncalibrated"
        rec = dict(s, fetch_kb_raw=f, fetch_correction=cal, write_kb=w)
        if f is not None and w is not None:
            b = (f * fac + w) * 1024.0
            rec["hbm_bytes_per_dispatch"] = b
            rec["hbm_bytes_per_step"] = b * s["calls"] / float(iters)
        out[name] = rec
    os.makedirs(os.path.dirname(dst_prefix) or ".", exist_ok=True)
    json.dump(out, open(dst_prefix + "_pmc.json", "w"), indent=1, sort_keys=True)
    with open(ks) as fi, open(dst_prefix + "_kernel_stats.csv", "w") as fo:
        fo.write(fi.read())
    print(json.dumps({k: v for k, v in out.items() if k.startswith("k_")}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4])
