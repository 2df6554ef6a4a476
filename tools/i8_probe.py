"""Config-4 batched search with the f16 filter vs the int8 filter copy on one shard.

python tools/i8_probe.py [--rows N] [--queries Q] [--k K] [--reps R]
Prints one JSON line: per-filter ms per batch, filter TFLOP/s (TOP/s for int8), fallbacks,
candidates kept per query per stage are not exposed; identical = the two result sets match bit for bit.
"""
import argparse
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--queries", type=int, default=1024)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="f16 or i8: run one filter only")
    args = ap.parse_args()
    import torch

    index = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.index")
    d = index.DeviceIndex(512, dtype="float16", capacity=args.rows, device=0)
    d.fill_random(4, 0, args.rows)
    g = torch.Generator(device="cuda").manual_seed(6)
    q = torch.randn((args.queries, 512), device="cuda", generator=g)
    out = {"rows": args.rows, "queries": args.queries, "k": args.k}
    res = {}
    for tag in ("f16", "i8"):
        if args.only and tag != args.only:
            continue
        if tag == "i8":
            t0 = time.perf_counter()
            d.set_filter("i8")
            torch.cuda.synchronize()
            out["quantise_s"] = time.perf_counter() - t0
        res[tag] = d.search(q, args.k, args.rows, mode="mfma")
        torch.cuda.synchronize()
        d.timing(True)
        d.gemm_timing_read()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            res[tag] = d.search(q, args.k, args.rows, mode="mfma")
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.reps
        ms, n, fl, fb = d.gemm_timing_read()
        d.timing(False)
        out[tag] = {"ms_per_batch": el * 1e3, "queries_per_s": args.queries / el, "filter_ms_per_batch": ms / args.reps,
                    "filter_tops": fl / (ms / 1e3) / 1e12 if ms else 0, "launches": n, "fallbacks": fb}
        print(f"{tag}: {out[tag]}", file=sys.stderr, flush=True)
    if len(res) == 2:
        out["identical"] = bool(torch.equal(res["f16"][0], res["i8"][0]) and torch.equal(res["f16"][1], res["i8"][1]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
