"""Result writers vs the reference's own writers (tests/golden/make_writer_golden.py ran
whisperx/utils.py:171-431 on the reference align() results in align_cases.json, plus
speaker / untimed-word / long-pause / no-words variants, under five subtitle option sets).
Byte-exact file contents for txt, vtt, srt, tsv, json, aud."""
import copy
import gzip
import json
import os

import pytest

from conftest import GOLDEN
from whisperx_amd import writers

with gzip.open(os.path.join(GOLDEN, "writer_cases.json.gz"), "rt", encoding="utf-8") as f:
    DATA = json.load(f)


@pytest.mark.parametrize("ci", range(len(DATA["cases"])))
def test_writer_outputs_match_reference(ci, tmp_path):
    case = DATA["cases"][ci]
    for fmt, expected in case["outputs"].items():
        w = writers.get_writer(fmt, str(tmp_path))
        w(copy.deepcopy(case["result"]), "/some/dir/audio.wav", dict(case["options"]))
        got = (tmp_path / f"audio.{fmt}").read_text(encoding="utf-8")
        assert got == expected, f"{case['name']} {case['options']} {fmt}"


def test_format_timestamp_matches_reference():
    for c in DATA["format_timestamp"]:
        assert writers.format_timestamp(c["seconds"], c["always_include_hours"], c["decimal_marker"]) == c["out"]


def test_write_all(tmp_path):
    case = DATA["cases"][0]
    writers.get_writer("all", str(tmp_path))(copy.deepcopy(case["result"]), "x.mp3", dict(case["options"]))
    assert sorted(p.name for p in tmp_path.iterdir()) == ["x.json", "x.srt", "x.tsv", "x.txt", "x.vtt"]
