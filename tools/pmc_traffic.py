"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage:
    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        [--out profiles/pmc_traffic.json]

Counter values are in KiB (rocprofv3 derived metrics).  Corrections from
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read on gfx950, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  The edge
kernel (a pure 16-B/lane stream of a known 224.5 MB edge_attr) is the
calibration point and its ratio is printed.

The JSON maps bench.py's kernel_table names to per-launch bytes; bench.py
reads it into roofline.traffic.
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict

# bench.py kernel_table name -> rocprof kernel name (the C2 instantiation; round
# 5 added defaulted template parameters: k_gemm3d's B read distance, k_gemm_bw's
# wave grid, which now appear in the names)
KERNELS = {
    "gemm_l0_fwd": "sv2n::k_gemm3d<12, 1, 9, 2, false, 1, false, false>",  # round 6: 12 waves
    "gemm_l0_dwT": "sv2n::k_gemm_tt3y<13, 2, false>",
    "edge_logits_fwd": "sv2n::k_edge_fwd_mx<16>",
    "edge_logits_bwd": "sv2n::k_edge_bwd_mx<16, 1>",
    "gat_attn_fwd_l0": "sv2n::canon::k_fwd<1, true, false, false>",
    "gat_attn_bwd_l0": "sv2n::canon::k_bwd<0, true, false, 3>",
    "gat_attn_fwd_l1_head": "sv2n::canon::k_fwd<1, false, false, true>",
    # the covariance-layout passes the C2 step runs (bench kernel_table
    # edge_logits_fwd_cv / _bwd_cv); the backward's slab reduce shares its
    # kernel name with the generic pass's and is listed on its own
    "edge_logits_fwd_cv": "sv2n::k_edge_fwd_cv2<6, 8>",
    "edge_logits_bwd_cv": "sv2n::k_edge_bwd_cv2<2, 8>",
    "edge_reduce_partials": "sv2n::k_reduce_partials",
}


# C5 (tools/measure.sh pmc): keys prefixed "c5:" in the same JSON
KERNELS_C5 = {
    "gat_attn_fused_fwd_l0": "sv2n::fused::k_fattn_fwd<12, false, false>",
    "gat_attn_fused_bwd_l0": "sv2n::fused::k_fattn_bwd2<12, false, false>",
    "gemm_l0_fwd": "sv2n::k_gemm3d<12, 1, 9, 2, false, 1, false, false>",
}

# C3 bf16 loop (tools/measure.sh pmc): keys "c3_bf16:..."; a list sums its kernels
# (the weight-gradient node is the GEMM and its epilogue launch)
KERNELS_C3 = {
    "gemm_fwd": "sv2n::k_gemm_bw<256, 192, false, false, false, 2, 4, 64>",  # a16: bf16 x twin
    "wgrad_node": ["sv2n::k_gemm_bw<128, 128, true, false, false, 2, 4, 64>", "sv2n::k_wgrad_epi_t"],
    "gat_attn_fwd": "sv2n::canon::k_fwd<1, false, false, false>",
    "gat_attn_bwd": "sv2n::canon::k_bwd<1, false, false, 2>",
    "window_gather": "sv2n::k_window_rows",
    "head_mse_train": "sv2n::k_head_mse_train_w<1, 8, true>",
}


def per_kernel(path, counter):
    """mean over dispatches of the dispatch's counter sum (KiB), keyed by kernel name."""
    disp = defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        disp[d] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    acc = defaultdict(list)
    for d, v in disp.items():
        acc[name[d]].append(v)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def find(table, prefix):
    if isinstance(prefix, list):
        parts = [find(table, p) for p in prefix]
        if any(p is None for p in parts):
            return None
        return (sum(p[0] for p in parts), min(p[1] for p in parts))
    for k, v in table.items():
        if prefix + "(" in k:
            return v
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--config", default="c2", choices=("c2", "c5", "c3_bf16"))
    a = ap.parse_args()
    fetch = per_kernel(a.fetch, "FETCH_SIZE")
    write = per_kernel(a.write, "WRITE_SIZE")
    out = {}
    try:
        out = json.load(open(a.out))  # merge: C2 and C5 passes share the file
    except (OSError, ValueError):
        pass
    out["_note"] = ("hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), "
                    "gfx950 FETCH_SIZE halving corrected per MI355X_MICROARCH.md; mean over "
                    "the dispatches of the profiled C2 train/forward steps (keys 'c5:...': "
                    "the C5 steps)")
    table = KERNELS if a.config == "c2" else \
        {a.config + ":" + k: v for k, v in (KERNELS_C5 if a.config == "c5" else KERNELS_C3).items()}
    for key, prefix in table.items():
        f, w = find(fetch, prefix), find(write, prefix)
        if f is None or w is None:
            continue
        fb, wb = 2.0 * f[0] * 1024.0, w[0] * 1024.0
        out[key] = {"kernel": " + ".join(prefix) if isinstance(prefix, list) else prefix,
                    "fetch_bytes": round(fb), "write_bytes": round(wb),
                    "hbm_bytes_per_launch": round(fb + wb), "dispatches": f[1]}
        print(f"{key:26s} read {fb / 1e6:9.2f} MB  write {wb / 1e6:8.2f} MB  ({f[1]} dispatches)")
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
