"""GEMM lab driver (diagnostic): time lab.hip's main-loop variants on the ViT-MSN batch-256
shapes, interleaved in one process, next to the vendor GEMM (torch.mm -> hipBLASLt) as a
yardstick; check every variant bit-identical to variant 0 and variant 0 against torch.
Variant 1's per-barrier s_memtime stamps are summarised per segment.

usage: python tools/gemm_lab/lab.py [--variants 0,2,3,4] [--rounds 5] [--stamps]
(build: hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -shared lab.hip -o liblab.so)
"""
import argparse
import ctypes as C
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SHAPES = {"qkv": (2304, 768), "o": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,2,3,4,5,6,16,32,48,64")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--shapes", default="qkv,o,fc1,fc2")
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--groups", default="", help="tile-order sweep for variant 0: group_m values, e.g. 0,2,4,8,16")
    args = ap.parse_args()
    lib = C.CDLL(os.path.join(HERE, "liblab.so"))
    lib.lab_gemm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                             C.c_int]
    dev = torch.device("cuda", 0)
    M = args.images * 197
    Mp = (M + 255) // 256 * 256
    variants = [int(v) for v in args.variants.split(",")]
    stamps = torch.zeros(16 * 512, dtype=torch.int64, device=dev)
    out = {}
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(1)
        A = (torch.rand(Mp, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        Cs = {v: torch.zeros(M, N, dtype=torch.bfloat16, device=dev) for v in variants}
        s = torch.cuda.current_stream().cuda_stream

        def run(v, grp=-1):
            rc = lib.lab_gemm(v, A.data_ptr(), W.data_ptr(), Cs[v].data_ptr(), M, N, K, stamps.data_ptr(), s, grp)
            assert rc == 0, rc

        Am = A[:M]
        legs = {f"v{v}": (lambda v=v: run(v)) for v in variants}
        for grp in [int(x) for x in args.groups.split(",") if x.strip()]:
            legs[f"v{variants[0]}_g{grp}"] = lambda grp=grp: run(variants[0], grp)
        legs["vendor_mm"] = lambda: torch.mm(Am, W.t())
        times = {k: [] for k in legs}
        for _ in range(args.rounds):
            for k, fn in legs.items():
                for _ in range(2):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / args.reps * 1e3)
        flops = 2.0 * M * N * K
        ref = torch.mm(Am.float(), W.float().t())
        v0 = variants[0]
        err = ((Cs[v0].float() - ref).abs() / (ref.abs() + 1e-2)).max().item()
        res = {k: {"us_min": round(min(t), 2), "us_med": round(sorted(t)[len(t) // 2], 2),
                   "TFLOPs": round(flops / (min(t) * 1e-6) / 1e12, 1)} for k, t in times.items()}
        res["check"] = {"v%d_vs_torch_max_rel" % v0: err,
                        "bit_identical": {f"v{v}": bool(torch.equal(Cs[v], Cs[v0])) for v in variants if v < 16}}
        print(name, json.dumps(res), flush=True)
        out[name] = res
        if args.stamps:
            lib.lab_gemm(1, A.data_ptr(), W.data_ptr(), Cs[v0].data_ptr(), M, N, K, stamps.data_ptr(), s, -1)
            torch.cuda.synchronize()
            st = stamps.view(16, 512).cpu()
            nk = K // 64
            # stamps per group: [entry, after prologue barrier, then per K-step per phase: after M
            # barrier, after C barrier] ...; segment lengths in cycles
            for grp in (0, 1):
                segs = []
                for b in range(8):
                    row = st[b * 2 + grp]
                    n = int((row != 0).sum())
                    d = (row[1:n] - row[: n - 1]).tolist()
                    segs.append(d)
                # K-loop part: d[1 .. 1 + 8 nk): alternate M->C (C segment incl. barrier), C->M
                per = [[0.0] * 8 for _ in range(1)]
                tot = [0.0] * 8
                cnt = 0
                for d in segs:
                    body = d[1:1 + 8 * nk]
                    if len(body) < 8 * nk:
                        continue
                    for kt in range(1, nk):  # skip the first K-step
                        for j in range(8):
                            tot[j] += body[8 * kt + j]
                    cnt += nk - 1
                avg = [round(t / max(cnt, 1), 1) for t in tot]
                first = [round(sum(d[0] for d in segs) / len(segs), 1)]
                tail = [round(sum(sum(d[1 + 8 * nk:]) for d in segs) / len(segs), 1)]
                print(f"  stamps {name} grp{grp}: prologue {first} per-K-step segments (cycles) {avg} "
                      f"sum {round(sum(avg), 1)} tail {tail}", flush=True)
                out[name][f"stamps_grp{grp}"] = {"segments": avg, "sum": sum(avg)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
