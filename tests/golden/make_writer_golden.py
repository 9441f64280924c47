"""Golden outputs of the reference's result writers (whisperx/utils.py:171-431).

Runs in the build container only: loads /root/reference/whisperx/utils.py (stdlib imports
only) by path, feeds it the aligned results already stored in align_cases.json (themselves
produced by the reference's align()) plus speaker-labelled / no-words / ja variants, under
several subtitle option sets, and records every writer's file content.  Writes
writer_cases.json.gz (inputs + outputs, no reference source).

    python tests/golden/make_writer_golden.py
"""
import copy
import gzip
import importlib.util
import json
import os
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/whisperx/utils.py"


def load_reference_utils():
    spec = importlib.util.spec_from_file_location("ref_whisperx_utils", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def results():
    cases = json.load(open(os.path.join(HERE, "align_cases.json")))
    out = []
    for c in cases:
        r = copy.deepcopy(c["result"])
        r["language"] = c["lang"]
        out.append((f"align_{c['lang']}_{c['split']}", r))
    # speaker labels on every other segment, a word without timing, a pause > 3 s
    base = copy.deepcopy(out[0][1])
    for i, s in enumerate(base["segments"]):
        if i % 2 == 0:
            s["speaker"] = f"SPEAKER_{i:02d}"
    if base["segments"] and len(base["segments"][0]["words"]) > 2:
        w = base["segments"][0]["words"][1]
        for k in ("start", "end", "score"):
            w.pop(k, None)
    if len(base["segments"]) > 1:
        for w in base["segments"][-1]["words"]:
            for k in ("start", "end"):
                if k in w:
                    w[k] = round(w[k] + 5.0, 3)
    out.append(("speakers_untimed_pause", base))
    # segments without words (e.g. a transcription result), tabs/arrows in text
    plain = {"language": "en", "segments": [
        {"start": 0.0, "end": 2.5, "text": " first\tline --> here "},
        {"start": 3661.25, "end": 3662.0005, "text": "second", "speaker": "SPEAKER_01"},
        {"start": 7.0015, "end": 9.9995, "text": "third "},
    ]}
    out.append(("no_words", plain))
    return out


OPTIONS = [
    {"max_line_width": None, "max_line_count": None, "highlight_words": False},
    {"max_line_width": None, "max_line_count": None, "highlight_words": True},
    {"max_line_width": 20, "max_line_count": 2, "highlight_words": False},
    {"max_line_width": 12, "max_line_count": 1, "highlight_words": True},
    {"max_line_width": 42, "max_line_count": None, "highlight_words": False},
]
FORMATS = ["txt", "vtt", "srt", "tsv", "json", "aud"]


def main():
    utils = load_reference_utils()
    cases = []
    with tempfile.TemporaryDirectory() as tmp:
        for name, res in results():
            for oi, opt in enumerate(OPTIONS):
                outs = {}
                for fmt in FORMATS:
                    writer = utils.get_writer(fmt, tmp)
                    writer(copy.deepcopy(res), os.path.join(tmp, "audio.wav"), dict(opt))
                    with open(os.path.join(tmp, "audio." + fmt), encoding="utf-8") as f:
                        outs[fmt] = f.read()
                cases.append({"name": name, "options": opt, "result": res, "outputs": outs})
        ts = [(s, h, m) for s in (0.0, 0.0004, 0.0005, 0.0015, 59.9995, 61.25, 3599.9996, 3723.4567, 86400.5)
              for h in (False, True) for m in (".", ",")]
        stamps = [{"seconds": s, "always_include_hours": h, "decimal_marker": m,
                   "out": utils.format_timestamp(s, h, m)} for s, h, m in ts]
    with gzip.open(os.path.join(HERE, "writer_cases.json.gz"), "wt", encoding="utf-8") as f:
        json.dump({"cases": cases, "format_timestamp": stamps}, f, ensure_ascii=False)
    print(len(cases), "writer cases,", len(stamps), "timestamps")


if __name__ == "__main__":
    main()
