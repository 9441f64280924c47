"""Untrained-Punkt sentence spans (whisperx_amd/punkt.py), used by align() when nltk is
absent (alignment.py:169-172 with PUNKT_ABBREVIATIONS).  nltk is not installed, so parity
with it is unpinned; these expectations were checked by hand against the nltk 3.8.1
algorithm (break after a period-final non-abbreviation followed by a token; abbreviations and
initials never break; closing quotes realigned into the sentence)."""
import pytest

from whisperx_amd.alignment import PUNKT_ABBREVIATIONS
from whisperx_amd.punkt import span_tokenize

CASES = [
    ("Hello world. This is a test.", ["Hello world.", "This is a test."]),
    ("Dr. Smith went home. He slept.", ["Dr. Smith went home.", "He slept."]),
    ("Mr. Brown vs. Mrs. Green. Prof. X won.", ["Mr. Brown vs. Mrs. Green.", "Prof. X won."]),
    ("It costs 3.5 dollars. Yes it does.", ["It costs 3.5 dollars.", "Yes it does."]),
    ("Wait... what? No! Never.", ["Wait... what?", "No!", "Never."]),
    ('He said "stop." Then he left.', ['He said "stop."', "Then he left."]),
    ("I met J. K. Rowling. she smiled.", ["I met J. K. Rowling.", "she smiled."]),
    ("The year 1999. It was good.", ["The year 1999.", "It was good."]),
    ("No punctuation at all", ["No punctuation at all"]),
    ("  leading spaces. trailing   ", ["  leading spaces.", "trailing"]),
    ("one.two. three", ["one.two.", "three"]),
    ("Ends with a period.", ["Ends with a period."]),
    ("", []),
]


@pytest.mark.parametrize("text,sentences", CASES)
def test_span_tokenize_hand_checked(text, sentences):
    spans = span_tokenize(text, PUNKT_ABBREVIATIONS)
    assert [text[a:b] for a, b in spans] == sentences
    assert all(0 <= a < b <= len(text) for a, b in spans)
    assert spans == sorted(spans)


def test_abbreviation_set_matters():
    t = "Dr. Smith arrived. Fine."
    assert len(span_tokenize(t, PUNKT_ABBREVIATIONS)) == 2
    assert len(span_tokenize(t, [])) == 3  # without the abbreviation "Dr." ends a sentence


def test_align_uses_restated_splitter_without_nltk():
    from whisperx_amd import alignment

    alignment._punkt = None
    try:
        assert alignment._sentence_spans("Hello there. General Kenobi.") == [(0, 12), (13, 28)]
    finally:
        alignment._punkt = None
