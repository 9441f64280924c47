"""Per-kernel roofline of the VAD producer (vad.py:198-240: pyannote's PyanNet segmentation
forward over 5 s windows every 0.5 s, then the overlap-add) over one hour of audio (development
tool; VERDICT round 5, Next #6): from a rocprofv3 kernel trace of `tools/legs.py vad1h`, the
LAST hour's kernels by category with the category's algorithmic FLOP and HBM bytes for that
hour, its summed kernel time, TFLOP/s and fraction of the 157.3 TFLOP/s fp32 MFMA peak, or
GB/s and fraction of 8 TB/s for the memory-bound stages.

PyanNet geometry per 5 s window (80,000 samples): sinc filterbank 80 x 251 taps, stride 10 ->
7,975 frames -> |.|, max-pool 3 -> 2,658; conv 80 -> 60, k 5 -> 2,654 -> pool -> 884; conv
60 -> 60, k 5 -> 880 -> pool -> 293; 2-layer bidirectional LSTM (H 128) over 293 steps; linear
256 -> 128 -> 128; classifier 128 -> 3.  The sinc filterbank runs once over the waveform
(windows overlap tenfold), so its FLOPs are those of 5.76 M frames, not 7,191 x 7,975.

    python tools/vad_roofline.py TRACE.csv [--out profiles/r6_vad_roofline.json]
"""
import argparse
import csv
import json

PEAK_TFLOPS = 157.3
PEAK_GBPS = 8000.0
WIN = 7191            # windows in one hour (5 s every 0.5 s, last one zero-padded)
F_SINC = 3600 * 16000 // 10  # sinc filterbank output frames over the hour (stride 10)
L1, P1, L2, P2, L3, P3 = 7975, 2658, 2654, 884, 880, 293
H = 128
f4 = 4


def per_hour():
    lstm_in = 2 * P3 * (60 * 8 * H + 2 * H * 8 * H)          # x W_ih^T for both layers, both directions
    lstm_rec = 2 * 2 * P3 * 4 * H * H * 2                    # h W_hh^T: 2 layers x 2 directions
    return {
        "sinc_filterbank_gemm": (2 * F_SINC * 80 * 251, f4 * (F_SINC * 10 + F_SINC * 80)),
        "sincnet_stage_epilogues": (0, f4 * WIN * (L1 * 80 + P1 * 80 + L2 * 60 + P2 * 60 + L3 * 60 + P3 * 60)),
        "conv_taps_80to60": (WIN * 2 * L2 * 60 * 80 * 5, f4 * WIN * (P1 * 80 + L2 * 60)),
        "conv_taps_60to60": (WIN * 2 * L3 * 60 * 60 * 5, f4 * WIN * (P2 * 60 + L3 * 60)),
        "lstm_input_gemms": (WIN * lstm_in, f4 * WIN * P3 * (60 + 256 + 2 * 8 * H)),
        "lstm_recurrence": (WIN * lstm_rec, f4 * WIN * P3 * (2 * 8 * H + 2 * 2 * H)),
        "linear_classifier_gemms": (WIN * 2 * P3 * (256 * 128 + 128 * 128 + 128 * 3), f4 * WIN * P3 * (256 + 2 * 128 + 3)),
        "overlap_add": (0, f4 * (WIN * P3 * 3 + 213_333)),
    }


def classify(n):
    if "sinc_stage" in n:
        return "sincnet_stage_epilogues"
    if "conv_taps_kernel<80" in n:
        return "conv_taps_80to60"
    if "conv_taps_kernel<64" in n:
        return "conv_taps_60to60"
    if "lstm_layer" in n:
        return "lstm_recurrence"
    if "vad_aggregate" in n:
        return "overlap_add"
    if "sinc_fb_kernel" in n or n.startswith("Cijk_Ailk"):  # (wx_sinc_filterbank; before it the unfold GEMM)
        return "sinc_filterbank_gemm"
    if "MT256x256" in n:
        return "lstm_input_gemms"
    if n.startswith("Cijk_"):
        return "linear_classifier_gemms"
    return "glue (norms of the waveform, activations, copies, fills)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    agg = [i for i, r in enumerate(rows) if "vad_aggregate" in r["Kernel_Name"]]
    start, end = agg[-2] + 1, agg[-1]  # the last hour: after the previous hour's overlap-add
    cat = {}
    for r in rows[start:end + 1]:
        k = classify(r["Kernel_Name"])
        e = cat.setdefault(k, {"calls": 0, "us": 0.0})
        e["calls"] += 1
        e["us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    span = (int(rows[end]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3
    ph = per_hour()
    out = {"source": a.trace, "audio": "1 h, 7,191 windows (PyanNet shape, random weights), fp32",
           "peak_tflops_fp32_mfma": PEAK_TFLOPS, "peak_hbm_GBps": PEAK_GBPS, "hour_span_us": round(span, 1),
           "categories": {}}
    tot_us = tot_flop = 0.0
    for k, e in sorted(cat.items(), key=lambda kv: -kv[1]["us"]):
        flop, byt = ph.get(k, (0, 0))
        us = e["us"]
        tot_us += us
        tot_flop += flop
        rec = {"calls": e["calls"], "kernel_us": round(us, 1), "gflop": round(flop / 1e9, 1), "mbytes": round(byt / 1e6, 1)}
        if flop:
            rec["tflops"] = round(flop / us / 1e6, 1)
            rec["frac_fp32_mfma_peak"] = round(flop / us / 1e6 / PEAK_TFLOPS, 3)
        if byt:
            rec["GBps"] = round(byt / us / 1e3, 1)
            rec["frac_hbm"] = round(byt / us / 1e3 / PEAK_GBPS, 3)
        rec["bound"] = "mfma" if flop and flop / max(byt, 1) > 20 else "hbm"
        out["categories"][k] = rec
    out["producer_kernel_us"] = round(tot_us, 1)
    out["producer_gflop"] = round(tot_flop / 1e9, 1)
    out["producer_tflops"] = round(tot_flop / tot_us / 1e6, 1)
    out["producer_frac_fp32_mfma_peak"] = round(tot_flop / tot_us / 1e6 / PEAK_TFLOPS, 3)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
