"""profiles/pmc_conv_latest.json (the traffic bench.py reports as roofline.traffic) from a roofline summary written by
tools/roofline_from_trace.py with --fetch / --write PMC passes.  usage: python tools/pmc_latest.py ROOFLINE.json TAG"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, tag = sys.argv[1], sys.argv[2]
r = json.load(open(src))
p = r["pmc"]
out = {
    "family": "KWS bf16 conv family of the timed steps: conv_igemm* (incl. conv_igemm_p8) + conv_ring + conv_stream + "
              "bottleneck_kernel on the scoring streams (encoder GEMMs and the compensated re-scoring tier excluded; "
              "tools/roofline_from_trace.py)",
    "launches_per_step": r["kws_conv_launches_per_step"],
    "fetch_bytes_per_step": p["fetch_bytes_per_step"],
    "write_bytes_per_step": p["write_bytes_per_step"],
    "bytes_per_step": p["bytes_per_step"],
    "bytes_per_launch": p["bytes_per_launch"],
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes of bench.py --steps 3 --warmup 1 ({tag}), "
              "records cut to the timed region by bench.py --prof-dump's CLOCK_MONOTONIC bounds; " + p["correction"],
}
# the isolated per-kernel table travels beside it (profiles/r0* stays off the GPU box): bench.py's
# roofline.per_kernel_isolated
if r.get("per_kernel_isolated"):
    with open(os.path.join(REPO, "profiles", "isolated_latest.json"), "w") as f:
        json.dump({"source": f"{src} per_kernel_isolated ({tag}: the rocprofv3 --pmc FETCH_SIZE pass, kernels serialised)",
                   "per_kernel_isolated": r["per_kernel_isolated"]}, f, indent=1)
        f.write("\n")
with open(os.path.join(REPO, "profiles", "pmc_conv_latest.json"), "w") as f:
    json.dump(out, f, indent=1)
    f.write("\n")
print(json.dumps(out, indent=1))
