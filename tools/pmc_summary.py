"""Summarise rocprofv3 --pmc passes (tools/run_pmc.sh) for hnsw_search_kernel into a traffic
record bench.py reports as roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) counts 128 B requests as 64 B for
wide coalesced reads -> bytes_read = 2 * FETCH_SIZE * 1024 (cross-checked: TCC_EA0_RDREQ_sum * 64
equals FETCH_SIZE * 1024 when TCC_EA0_RDREQ_32B_sum == 0).  WRITE_SIZE (KB) is taken as is.
usage: python tools/pmc_summary.py gpurun_out profiles/r01/traffic.json [flat]
  (flat: tools/run_pmc_flat.sh's flat scan kernel passes; algorithmic bytes = the base read once)
"""

import csv
import glob
import json
import os
import re
import sys


def per_launch(path, kernel="hnsw_search_kernel"):
    vals = {}
    names = set()
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            names.add(re.search(r"\w*" + kernel + r"\w*", r["Kernel_Name"]).group(0))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, names


def main(src, dst, mode="hnsw"):
    c = {}
    launches = {}
    # flat: whichever scan kernel the dispatch picked (flat_scan_kernel / _ws_kernel / _wide_kernel)
    prefix, kernel = ("pmcf_", "flat_scan_") if mode == "flat" else ("pmc_", "hnsw_search_kernel")
    names = set()
    for f in glob.glob(os.path.join(src, prefix + "*", "run_counter_collection.csv")):
        v, n, nm = per_launch(f, kernel)
        c.update(v)
        launches.update(n)
        names |= nm
    if len(names) > 1:
        sys.exit(f"passes profiled different kernels: {sorted(names)}")
    cfg = json.load(open(os.path.join(src, prefix + "FETCH_SIZE.json")))
    read_b = 2.0 * c["FETCH_SIZE"] * 1024.0
    write_b = c.get("WRITE_SIZE", 0.0) * 1024.0
    if mode == "flat":  # the base and the queries read once, the chunk shortlists written once
        cf = cfg["config"]
        alg = 4.0 * cf["dim"] * (cf["n_base"] + cf["n_queries"]) + 4.0 * cf["n_base"]
        if any("tiles" in n for n in names):  # the single-role scan reads the f16 tile records instead
            k = (cf["dim"] + 31) // 32 * 32
            alg = (cf["n_base"] + 31) // 32 * (k // 16 * 1024 + 256) + 4.0 * cf["dim"] * cf["n_queries"]
    else:
        alg = cfg["roofline"]["algorithmic_bytes_per_launch"]
        if cfg.get("dtype") == "u8+f32":  # SQ8: the profiled kernel is the search; the rerank's f32 rows
            cf = cfg["config"]            # (k + 1 per query, bench.py) belong to rerank_kernel
            alg -= 4.0 * cf["dim"] * (cf["k"] + (1 if cf["ef_search"] > cf["k"] else 0)) * cf["n_queries"]
    hit = c.get("TCC_HIT_sum", 0.0)
    miss = c.get("TCC_MISS_sum", 0.0)
    out = {
        "kernel": names.pop() if names else kernel,
        "config": {k: cfg["config"][k] for k in ("workload", "n_base", "n_queries", "dim", "k", "ef_search")
                   if k in cfg["config"]},
        "launches_per_pass": launches,
        "counters_per_launch": c,
        "hbm_read_bytes_per_launch": read_b,
        "hbm_write_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "rdreq_x64_over_fetch": (c.get("TCC_EA0_RDREQ_sum", 0.0) * 64.0) / (c["FETCH_SIZE"] * 1024.0)
        if "TCC_EA0_RDREQ_sum" in c else None,
        "profiled_kernel_ms": cfg["roofline"]["kernel_ms"],
    }
    if mode == "flat":  # the shortlist contraction the profiled scan ran (bench.py's roofline.contraction)
        out["contraction"] = cfg["roofline"].get("contraction", "bf16x3")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=2)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
