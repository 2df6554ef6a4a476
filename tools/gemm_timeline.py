"""Per-workgroup phase timeline of the projection GEMMs (diagnostic build: tools/build_diag.sh).

The diag kernels stamp s_memrealtime (100 MHz) at: workgroup entry, K loop start (after the
prologue DMA wait), K loop end, epilogue end (gemm_pp_kernel), or per segment of a stream-K
workgroup.  For each shape and variant: kernel span, per-phase medians, and how busy the CUs
are over time.   RC_LIB_PATH=...lib/diag/libretrieval_core.so python tools/gemm_timeline.py
"""
import ctypes as C
import importlib
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

L = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib")
lib = L.load()
raw = C.CDLL(L.LIB_PATH)
raw.rc_diag_set_stamps.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
M = 256 * 197
shapes = {"oproj": (768, 768, 2), "fc2": (768, 3072, 2), "qkv": (2304, 768, 0), "fc1": (3072, 768, 1)}
variants = [int(v) for v in os.environ.get("VARIANTS", "4").split(",")]
sel = os.environ.get("SHAPES", "oproj,fc2").split(",")
stamps = torch.zeros(4096 * 64, dtype=torch.int64, device=dev)
TICK_US = 0.01


def med(x):
    return float(np.median(x)) if len(x) else 0.0


out = {}
for name in sel:
    N, K, epi = shapes[name]
    Mp = (M + 255) // 256 * 256
    A = (torch.randn(Mp, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    o = torch.zeros(Mp, N, device=dev) if epi == 2 else torch.zeros(Mp, N, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    for v in variants:
        for _ in range(3):
            L.check(lib.rc_gemm_bf16(epi, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, o.data_ptr(), None, 0, s))
        torch.cuda.synchronize()
        stamps.zero_()
        L.check(raw.rc_diag_set_stamps(C.c_void_p(stamps.data_ptr())))
        L.check(lib.rc_gemm_bf16(epi, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, o.data_ptr(), None, 0, s))
        torch.cuda.synchronize()
        L.check(raw.rc_diag_set_stamps(None))
        st = stamps.cpu().numpy().reshape(-1, 64).astype(np.int64)
        used = st[(st[:, 0] != 0) | (st[:, 63] != 0)]
        res = {}
        if v == 4:
            t0, t1, t2, t3 = used[:, 0], used[:, 1], used[:, 2], used[:, 3]
            base = t0.min()
            res["span_us"] = (t3.max() - base) * TICK_US
            res["wgs"] = int(len(used))
            res["prologue_us"] = med((t1 - t0) * TICK_US)
            res["loop_us"] = med((t2 - t1) * TICK_US)
            res["epilogue_us"] = med((t3 - t2) * TICK_US)
            cu = defaultdict(list)
            for r in used:
                cu[(int(r[4]) >> 32, (int(r[4]) >> 8) & 0xFF, (int(r[4]) >> 13) & 0x7)].append(r)
            gaps = []
            for lst in cu.values():
                lst.sort(key=lambda r: r[0])
                for p, q in zip(lst, lst[1:]):
                    gaps.append((q[0] - p[3]) * TICK_US)
            res["cus"] = len(cu)
            res["dispatch_gap_us"] = med(gaps)
            res["rounds_first_entry_us"] = sorted(set(round((x - base) * TICK_US) for x in t0))[:3]
        else:
            base = None
            segs = []
            for r in used:
                for k in range(7):
                    q = r[8 * k: 8 * k + 8]
                    if q[0] == 0:
                        continue
                    segs.append((q[0], q[1], q[2], q[3], int(q[4]) >> 32, int(q[5]) & 0xFFFFFFFF, int(q[5]) >> 32))
            segs = np.array(segs, dtype=np.int64)
            base = segs[:, 0].min()
            res["span_us"] = (segs[:, 3].max() - base) * TICK_US
            res["wgs"] = int(len(used))
            for kind in (0, 1, 2):
                ss = segs[segs[:, 4] == kind]
                if len(ss) == 0:
                    continue
                steps = ss[:, 6] - ss[:, 5]
                res[f"kind{kind}"] = {"n": int(len(ss)), "prologue_us": med((ss[:, 1] - ss[:, 0]) * TICK_US),
                                      "loop_us_per_step": med((ss[:, 2] - ss[:, 1]) * TICK_US / np.maximum(steps, 1)),
                                      "tail_us": med((ss[:, 3] - ss[:, 2]) * TICK_US)}
            ends = np.sort((used[:, :56].reshape(-1, 7, 8)[:, :, 3].max(axis=1) - base) * TICK_US)
            res["wg_end_us_p10_p50_p90"] = [float(np.percentile(ends, p)) for p in (10, 50, 90)]
        out[f"{name}/{v}"] = res
        print(name, v, json.dumps(res), flush=True)
