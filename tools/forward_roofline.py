"""Per-kernel roofline of the wav2vec2-base emission forward inside align() (development tool;
VERDICT round 4, Next #2): from a rocprofv3 kernel trace of `tools/legs.py e2e` (16 x 30 s
segments per align() call), the LAST complete align() call's kernels by category, with the
category's algorithmic FLOP and HBM bytes for that call, its summed kernel time, TFLOP/s and
fraction of the 157.3 TFLOP/s fp32 MFMA peak (256 CUs x 4 SIMDs x 64 FLOP/clk x 2.4 GHz).

The packed encoder runs every kernel of a pack on one stream (emission.packed_logits), so the
durations are single-stream kernel times (only the DP of the previous pack may overlap).

    python tools/forward_roofline.py TRACE.csv [--segments 16] [--out profiles/r5_forward_roofline.json]
"""
import argparse
import csv
import json

PEAK_TFLOPS = 157.3
PEAK_GBPS = 8000.0

# wav2vec2-base over one 30 s segment (480,000 samples): frame counts per feature-encoder layer
L = [95999, 47999, 23999, 11999, 5999, 2999, 1499]
KS = [(3, 2)] * 4 + [(2, 2)] * 2
C, D, FF, H, V, NL = 512, 768, 3072, 12, 32, 12
T = L[-1]


def per_segment():
    """category -> (FLOP, HBM bytes) for one segment (algorithmic: each operand read once,
    each result written once)."""
    f = 4
    conv_flop = sum(2 * L[i + 1] * C * C * k for i, (k, _) in enumerate(KS))
    conv_bytes = sum(f * (L[i] * C + L[i + 1] * C + k * C * C) for i, (k, _) in enumerate(KS))
    gelu_fe_bytes = sum(2 * f * L[i + 1] * C for i in range(6))
    lay = {
        "qkv_gemm": (2 * T * D * 3 * D, f * (T * D + 3 * D * D + T * 3 * D)),
        "attention": (4 * T * T * 64 * H, f * (3 * T * D + T * D)),
        "out_proj_gemm": (2 * T * D * D, f * (2 * T * D + D * D)),
        "ff1_gemm": (2 * T * D * FF, f * (T * D + D * FF + T * FF)),
        "ff_gelu": (0, 2 * f * T * FF),
        "ff2_gemm": (2 * T * FF * D, f * (T * FF + FF * D + T * D)),
        "add_layernorm": (0, 2 * 3 * f * T * D),
    }
    out = {
        "conv0_norm_gelu": (2 * L[0] * C * 10, f * (480000 + L[0] * C)),
        "fe_conv_gemms": (conv_flop, conv_bytes),
        "fe_gelu": (0, gelu_fe_bytes),
        "feature_projection": (2 * T * C * D, f * (2 * T * C + C * D + T * D)),
        "posconv": (2 * T * D * (D // 16) * 128, f * (2 * T * D + D * (D // 16) * 128)),
        "lm_head_log_softmax": (2 * T * D * V, f * (T * D + 2 * T * V)),
    }
    for k, (a, b) in lay.items():
        out[k] = (NL * a, NL * b)
    return out


def classify(name, state):
    n = name
    if "conv0_" in n:
        return "conv0_norm_gelu"
    if "posconv" in n:
        state["enc"] = True
        state["alik"] = 0
        return "posconv"
    if "attn_f32" in n:
        return "attention"
    if "add_ln" in n:
        return "add_layernorm"
    if "Gelu" in n:
        return "ff_gelu" if state.get("enc") else "fe_gelu"
    if "softmax" in n:
        state["enc"] = False
        return "lm_head_log_softmax"
    if "align_dp" in n:
        return "dp (overlapping)"
    if n.startswith("Cijk_Ailk"):
        return "fe_conv_gemms"
    if n.startswith("Cijk_Alik"):
        if not state.get("enc"):
            return "feature_projection"
        i = state["alik"]
        state["alik"] = i + 1
        if i >= 4 * NL:
            return "lm_head_log_softmax"
        return ("qkv_gemm", "out_proj_gemm", "ff1_gemm", "ff2_gemm")[i % 4]
    if "layer_norm" in n:
        return "layernorm (projection / encoder)"
    return "glue (copies, fills, gathers)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--segments", type=int, default=16)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    # the last align() call: from the first conv0 kernel after the second-to-last DP launch group
    sm = [i for i, r in enumerate(rows) if "softmax" in r["Kernel_Name"]]
    c0 = [i for i, r in enumerate(rows) if "conv0_stats" in r["Kernel_Name"]]
    end = max(i for i, r in enumerate(rows) if "align_dp" in r["Kernel_Name"])
    # conv0 launches of the last call: the last `segments` conv0_stats kernels
    start = c0[-a.segments]
    state = {}
    cat = {}
    for r in rows[start:end + 1]:
        k = classify(r["Kernel_Name"], state)
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        e = cat.setdefault(k, {"calls": 0, "us": 0.0})
        e["calls"] += 1
        e["us"] += d
    wall = (int(rows[end]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3
    ps = per_segment()
    out = {"source": a.trace, "segments": a.segments, "model": "wav2vec2-base (random weights), 30 s segments, fp32",
           "peak_tflops_fp32_mfma": PEAK_TFLOPS, "peak_hbm_GBps": PEAK_GBPS,
           "call_span_us": round(wall, 1), "categories": {}}
    tot_us = tot_flop = 0.0
    for k, e in sorted(cat.items(), key=lambda kv: -kv[1]["us"]):
        flop, byt = ps.get(k, (0, 0))
        flop *= a.segments
        byt *= a.segments
        us = e["us"]
        tot_us += us if not k.startswith("dp") else 0.0
        tot_flop += flop
        rec = {"calls": e["calls"], "kernel_us": round(us, 1), "gflop": round(flop / 1e9, 2),
               "mbytes": round(byt / 1e6, 1)}
        if flop:
            rec["tflops"] = round(flop / us / 1e6, 1)
            rec["frac_fp32_mfma_peak"] = round(flop / us / 1e6 / PEAK_TFLOPS, 3)
        if byt:
            rec["GBps"] = round(byt / us / 1e3, 1)
            rec["frac_hbm"] = round(byt / us / 1e3 / PEAK_GBPS, 3)
        out["categories"][k] = rec
    out["forward_kernel_us"] = round(tot_us, 1)
    out["forward_gflop"] = round(tot_flop / 1e9, 1)
    out["forward_tflops"] = round(tot_flop / tot_us / 1e6, 1)
    out["forward_frac_fp32_mfma_peak"] = round(tot_flop / tot_us / 1e6 / PEAK_TFLOPS, 3)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
