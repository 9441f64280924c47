"""Sentence spans for align() without nltk (alignment.py:169-172).

The reference builds ``PunktSentenceTokenizer(PunktParameters())`` with only
``abbrev_types = {"dr", "vs", "mr", "mrs", "prof"}`` set -- no training data, so no
orthographic context, collocations or sentence starters -- and takes
``span_tokenize(text)`` of every segment.  nltk is not installed here or on the GPU box;
``align()`` uses the real tokenizer whenever nltk is importable and this restatement
otherwise.  It follows the published algorithm of nltk 3.8.1 (nltk/tokenize/punkt.py; the
reference's requirements.txt:7 leaves the version unpinned):

* candidate ends: ``[.?!]`` followed by a non-word punctuation mark or by whitespace and a
  token (``period_context_re``), each with the word before it as context
  (``_match_potential_end_contexts``);
* a candidate is a break when, in its context, a token annotated ``sentbreak`` is followed by
  another token (``text_contains_sentbreak``).  Annotation, first pass: ``.``/``?``/``!``
  tokens break; ``..``-runs are ellipses; a period-final token breaks unless its stem (or the
  stem's last ``-`` part) is an abbreviation.  Second pass, with empty orthographic context:
  an abbreviation or ellipsis never turns into a break (the orthographic heuristic can only
  say "lower case: no" or "unknown"); an initial (``X.``) or a number followed by a
  lower-case word (or ``;:,.!?``), and an initial followed by a capitalised word, are
  re-classified as non-breaks;
* ``_realign_boundaries`` moves closing quotes/brackets after a break into the sentence.

Spans are ``(start, end)`` character offsets, the next sentence starting at its first token.
Parity with nltk is **unpinned** (nltk absent: no fixture can be generated); the tests pin the
behaviour on hand-checked texts.
"""
from __future__ import annotations

import re
import string
from typing import Iterable, List, Optional, Tuple

_SENT_END = ".?!"
_NON_WORD = r"(?:[)\";}\]\*:@\'\({\[!?])"
_MULTI_CHAR = r"(?:\-{2,}|\.{2,}|(?:\.\s){2,}\.)"
_WORD_START = r"[^\(\"\`{\[:;&\#\*@\)}\]\-,]"

_WORD_TOKENIZE = re.compile(
    r"""(
        %(MultiChar)s
        |
        (?=%(WordStart)s)\S+?
        (?=
            \s|
            $|
            %(NonWord)s|%(MultiChar)s|
            ,(?=$|\s|%(NonWord)s|%(MultiChar)s)
        )
        |
        \S
    )""" % {"MultiChar": _MULTI_CHAR, "WordStart": _WORD_START, "NonWord": _NON_WORD},
    re.UNICODE | re.VERBOSE,
)
_PERIOD_CONTEXT = re.compile(
    r"""
    [%(SentEnd)s]
    (?=(?P<after_tok>
        %(NonWord)s
        |
        \s+(?P<next_tok>\S+)
    ))""" % {"SentEnd": re.escape(_SENT_END), "NonWord": _NON_WORD},
    re.UNICODE | re.VERBOSE,
)
_REALIGN = re.compile(r'["\')\]}]+?(?:\s+|(?=--)|$)', re.MULTILINE)
_NUMBER = re.compile(r"^-?[\.,]?\d[\d,\.-]*\.?$")
_ELLIPSIS = re.compile(r"\.\.+$")
_INITIAL = re.compile(r"[^\W\d]\.$", re.UNICODE)


class _Tok:
    __slots__ = ("tok", "type", "period_final", "sentbreak", "abbr", "ellipsis")

    def __init__(self, tok: str):
        self.tok = tok
        self.type = _NUMBER.sub("##number##", tok.lower())
        self.period_final = tok.endswith(".")
        self.sentbreak = False
        self.abbr = False
        self.ellipsis = False

    @property
    def type_no_period(self):
        return self.type[:-1] if len(self.type) > 1 and self.type[-1] == "." else self.type

    @property
    def first_upper(self):
        return self.tok[0].isupper()

    @property
    def first_lower(self):
        return self.tok[0].islower()


def _words(text: str) -> List[_Tok]:
    out = []
    for line in text.split("\n"):
        if line.strip():
            out += [_Tok(m.group(1)) for m in _WORD_TOKENIZE.finditer(line)]
    return out


def _ortho_heuristic(t: _Tok):
    """With no orthographic context (untrained parameters): False for punctuation and
    lower-case words, "unknown" otherwise (never True)."""
    if t.tok in ";:,.!?":
        return False
    if t.first_lower:
        return False
    return "unknown"


def _annotate(toks: List[_Tok], abbrevs) -> List[_Tok]:
    for t in toks:  # first pass
        if t.tok in _SENT_END:
            t.sentbreak = True
        elif _ELLIPSIS.match(t.tok):
            t.ellipsis = True
        elif t.period_final and not t.tok.endswith(".."):
            stem = t.tok[:-1].lower()
            if stem in abbrevs or stem.split("-")[-1] in abbrevs:
                t.abbr = True
            else:
                t.sentbreak = True
    for t1, t2 in zip(toks, toks[1:]):  # second pass (the last token has no successor)
        if not t1.period_final:
            continue
        if t1.abbr or t1.ellipsis:
            if _ortho_heuristic(t2) is True:  # unreachable without orthographic context
                t1.sentbreak = True
                continue
        if _INITIAL.match(t1.tok) or t1.type_no_period == "##number##":
            s = _ortho_heuristic(t2)
            if s is False or (s == "unknown" and _INITIAL.match(t1.tok) and t2.first_upper):
                t1.sentbreak = False
                t1.abbr = True
    return toks


def _contains_break(context: str, abbrevs) -> bool:
    found = False
    for t in _annotate(_words(context), abbrevs):
        if found:
            return True
        if t.sentbreak:
            found = True
    return False


def _end_contexts(text: str):
    prev_slice = (0, 0)
    prev_match = None
    for m in _PERIOD_CONTEXT.finditer(text):
        before = text[prev_slice[1]:m.start()]
        sp = max((i for i, c in enumerate(before) if c in string.whitespace), default=None)
        if sp:  # (nltk: a falsy index -- none, or 0 -- restarts at the previous word)
            start = sp + prev_slice[1] + 1
        else:
            start = prev_slice[0]
        word = (start, m.start())
        if prev_match is not None and prev_slice[1] <= word[0]:
            yield prev_match, text[prev_slice[0]:prev_slice[1]] + prev_match.group() + prev_match.group("after_tok")
        prev_match, prev_slice = m, word
    if prev_match is not None:
        yield prev_match, text[prev_slice[0]:prev_slice[1]] + prev_match.group() + prev_match.group("after_tok")


def _slices(text: str, abbrevs):
    last = 0
    for m, context in _end_contexts(text):
        if _contains_break(context, abbrevs):
            yield (last, m.end())
            last = m.start("next_tok") if m.group("next_tok") else m.end()
    yield (last, len(text.rstrip()))


def _realign(text: str, slices):
    slices = list(slices)
    realign = 0
    for i, (a, b) in enumerate(slices):
        a += realign
        if i + 1 == len(slices):
            if text[a:b]:
                yield (a, b)
            continue
        a2, b2 = slices[i + 1]
        m = _REALIGN.match(text[a2:b2])
        if m:
            yield (a, a2 + len(m.group(0).rstrip()))
            realign = m.end()
        else:
            realign = 0
            if text[a:b]:
                yield (a, b)


def span_tokenize(text: str, abbrev_types: Optional[Iterable[str]] = None) -> List[Tuple[int, int]]:
    """PunktSentenceTokenizer(params with abbrev_types).span_tokenize(text) for untrained
    parameters (nltk 3.8.1 algorithm, restated)."""
    abbrevs = set(abbrev_types or ())
    return list(_realign(text, _slices(text, abbrevs)))
