"""Per-phase time split of jpeg_band_resize_kernel (diagnostic; needs the diagnostic build,
RC_LIB_PATH=.../lib/diag/libretrieval_core.so, under rocprofv3 --kernel-trace): 256 fixture-shaped
JPEGs decoded with phase-skip masks (rc_diag_set_band_skip: 1 colour, 2 horizontal, 4 vertical
math, 8 plane copy, 16 vertical pass + stores skipped), REPS calls per mask in the order printed.  --parse <kernel_trace.csv> then folds
the band kernel's durations into per-mask medians.  RC_PHASE_MASKS=0,31 picks the masks."""
import importlib
import json
import os
import sys

MASKS = [int(x) for x in os.environ.get("RC_PHASE_MASKS", "0,1,2,4,3,7,15,31,32,64,72").split(",")]
REPS = 12

if len(sys.argv) > 2 and sys.argv[1] == "--parse":
    import csv

    rows = [r for r in csv.DictReader(open(sys.argv[2])) if "band_resize" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    d = d[-len(MASKS) * REPS:]
    out = {}
    for i, m in enumerate(MASKS):
        x = sorted(d[i * REPS + 2:(i + 1) * REPS])  # first two calls of a mask: warm-up
        out[f"skip{m}"] = round(x[len(x) // 2], 2)
    print(json.dumps({"band_kernel_us_median": out, "masks": "1 colour, 2 horizontal, 4 vertical math, 8 plane copy, 16 vertical pass + stores skipped, 32 return after descriptors, 64 return after plane DMA + taps"}))
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import synthetic_jpegs  # noqa: E402

J = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.jpeg")
lib = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib").load()
batch = synthetic_jpegs(256, 7100, size=(168, 300))
dec = J.JpegDecoder(device=0, max_images=256, max_pixels=256 * 168 * 304)
for m in MASKS:
    assert lib.rc_diag_set_band_skip(m) == 0
    for _ in range(REPS):
        dec.decode_resized(batch, 224, 3)
    torch.cuda.synchronize()
assert lib.rc_diag_set_band_skip(0) == 0
print(json.dumps({"masks": MASKS, "reps": REPS}), flush=True)
