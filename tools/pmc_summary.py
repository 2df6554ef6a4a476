"""Summarise rocprofv3 PMC passes (tools/pmc_collect.sh output) per kernel.

Per kernel (short name + grid size): mean counter values per dispatch, mean
duration, and derived numbers:
  hbm_read_bytes  = 2 * FETCH_SIZE * 1024   (gfx950: FETCH_SIZE reads half of a
                    wide coalesced stream — MI355X_MICROARCH.md §HBM; calibrate on
                    a known byte count before trusting absolutes)
  hbm_write_bytes = WRITE_SIZE * 1024
  l2_hit          = TCC_HIT / (TCC_HIT + TCC_MISS)
  mfma_busy       = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * CUs * 4 SIMDs)  (approx)
  clock_GHz       = GRBM_GUI_ACTIVE / 8 / duration
usage: python tools/pmc_summary.py DIR [--json OUT] [--latest profiles/pmc_latest.json]

--latest writes the per-launch HBM traffic of the kernels bench.py prices
(keys qkv, oproj, fc1, fc2, attention, patch, scan_f16, filter_f16, filter_i8),
averaged over that kernel's launches; --merge keeps entries this run did not launch.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("rc::", "")
    return name[:60]


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for key, cs in sorted(vals.items(), key=lambda kv: -sum(durs[kv[0]])):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        dur = sum(durs[key]) / len(durs[key])
        rec = {"kernel": key[0], "grid": key[1], "dispatches": max(len(v) for v in cs.values()), "dur_us": dur * 1e6}
        rec.update({c: m[c] for c in m})
        if "FETCH_SIZE" in m:
            rec["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            rec["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            rec["l2_hit"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if "GRBM_GUI_ACTIVE" in m:
            rec["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                rec["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"] > 0:
            # SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES count quad-cycles per wave: the share of wave lifetime
            # spent issuing each instruction class (VALU includes MFMA issue on gfx9 counters)
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    rec[c.replace("SQ_ACTIVE_INST_", "").lower() + "_issue_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_MFMA" in m:
            rec["valu_non_mfma_insts"] = m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]
        out[f"{key[0]}@{key[1]}"] = rec
    for k, r in out.items():
        if r["dur_us"] < 20:
            continue
        keys = ["dur_us", "hbm_read_bytes", "hbm_write_bytes", "l2_hit", "clock_GHz", "mfma_busy", "SQ_WAIT_ANY",
                "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "valu_issue_frac",
                "lds_issue_frac", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "valu_non_mfma_insts", "SQ_VALU_MFMA_COEXEC_CYCLES"]
        print(k, {x: (round(r[x], 3) if isinstance(r.get(x), float) else r.get(x)) for x in keys if x in r})
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    if "--latest" in sys.argv:
        # the model's projections (LayerNorm folded, bf16-pair residual stream): EPI 4 QKV,
        # 5 fc1, 6 O-proj (NKT 12) / fc2 (NKT 48)
        # (round 3: O-proj on the two-workgroup kernel; the int8 filter copy)
        keys = {"fc1": ("gemm_pp_kernel<5, 0, 12>",), "qkv": ("gemm_pp_kernel<4, 0, 12>",),
                "oproj": ("gemm_w2_kernel<6, 0>", "gemm_pp_kernel<6, 0, 12>"), "fc2": ("gemm_pp_kernel<6, 0, 48>",),
                "attention": ("attention_v2_kernel<197>",), "patch": ("patch_gemm_kernel<16, 7>",),
                "scan_f16": ("scan_topk_kernel<f16_t, 4, 1, 128>",),
                "filter_f16": ("filter_qs_kernel<f16_t, 8, 0>",), "filter_i8": ("filter_i8_kernel<4, 128>",)}
        latest = {}
        if "--merge" in sys.argv:  # keep the entries of kernels this run did not launch
            try:
                latest = json.load(open(sys.argv[sys.argv.index("--latest") + 1]))
            except (OSError, ValueError):
                latest = {}
        for key, knames in keys.items():
            # prefix match: "gemm_pp_kernel<5, 0, 12" also names the K-loop forms <5, 0, 12, KL>
            kname = next((k for k in knames if any(r["kernel"].startswith(k.rstrip(">")) for r in out.values())),
                         knames[0])
            recs = [r for r in out.values() if r["kernel"].startswith(kname.rstrip(">"))]
            if recs:  # bench prices the full-size launches (unsplit fc1, 125M-row scan / filter): the longest grid
                gmax = max(recs, key=lambda r: r["dur_us"])["grid"]
                recs = [r for r in recs if r["grid"] == gmax]
            if not recs or not all("hbm_read_bytes" in r and "hbm_write_bytes" in r for r in recs):
                continue
            n = sum(r["dispatches"] for r in recs)
            tot = sum((r["hbm_read_bytes"] + r["hbm_write_bytes"]) * r["dispatches"] for r in recs)
            latest[key] = {"kernel": kname, "dispatches": n, "hbm_bytes_per_launch": tot / n,
                           "hbm_read_bytes_per_launch": sum(r["hbm_read_bytes"] * r["dispatches"] for r in recs) / n,
                           "hbm_write_bytes_per_launch": sum(r["hbm_write_bytes"] * r["dispatches"] for r in recs) / n,
                           "note": "FETCH_SIZE x 2 (gfx950 wide-stream correction) + WRITE_SIZE, KiB units -> bytes"}
        json.dump(latest, open(sys.argv[sys.argv.index("--latest") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
