"""NLP tokenizers (upstream nlp/src/main/java/hivemall/nlp/tokenizer/
{KuromojiUDF,SmartcnUDF,TokenizeKoUDF}.java, StoptagsExcludeUDF).

Upstream wraps Lucene's Kuromoji / SmartCN / Nori analyzers, which need dictionaries that are
not available offline.  These functions keep the SQL surface with a dictionary-free
segmentation: text is split into runs of one script (Han, Hiragana, Katakana, Hangul, Latin
letters/digits); Hiragana runs that follow Han are attached to it (okurigana), and Han runs in
``tokenize_cn`` are split into overlapping bigrams (the classic CJK bigram analyzer).  Output is
deterministic; tokens differ from a morphological analyzer (docs/compat.md).
"""
from __future__ import annotations

import unicodedata

from ..registry import udf


def _script(ch: str) -> str:
    o = ord(ch)
    if 0x3040 <= o <= 0x309F:
        return "hira"
    if 0x30A0 <= o <= 0x30FF or 0x31F0 <= o <= 0x31FF or 0xFF66 <= o <= 0xFF9F:
        return "kata"
    if 0x4E00 <= o <= 0x9FFF or 0x3400 <= o <= 0x4DBF or 0xF900 <= o <= 0xFAFF:
        return "han"
    if 0xAC00 <= o <= 0xD7AF or 0x1100 <= o <= 0x11FF or 0x3130 <= o <= 0x318F:
        return "hangul"
    if ch.isalnum():
        return "latin"
    return "sep"


def _runs(text: str):
    text = unicodedata.normalize("NFKC", text)
    cur, kind = [], None
    for ch in text:
        k = _script(ch)
        if k == "sep":
            if cur:
                yield kind, "".join(cur)
            cur, kind = [], None
            continue
        if kind is None or k == kind or (kind == "han" and k == "hira"):
            cur.append(ch)
            kind = kind or k
        else:
            yield kind, "".join(cur)
            cur, kind = [ch], k
    if cur:
        yield kind, "".join(cur)


_JA_STOP = set("の に は を た が で て と し れ さ ある いる も する から な こと として い や れる など なっ ない この ため その あっ よう また もの という あり まで られ なる へ か だ これ によって により おり より による ず なり られる において ば なかっ なく しかし について せ だっ その後 できる それ う ので なお のみ でき き つ における および いう さらに でも ら たり その他 に関する たち ます ん なら".split())


@udf("tokenize_ja", "tokenize_ja_neologd")
def tokenize_ja(text, mode: str | None = None, stopwords=None, stoptags=None, userdict=None):
    if text is None:
        return None
    toks = [t for _, t in _runs(str(text))]
    stop = _JA_STOP if stopwords is None else set(stopwords)
    return [t for t in toks if t not in stop]


@udf("tokenize_cn")
def tokenize_cn(text, stopwords=None):
    if text is None:
        return None
    out = []
    for kind, t in _runs(str(text)):
        if kind == "han" and len(t) > 2:
            out.extend(t[i:i + 2] for i in range(len(t) - 1))
        else:
            out.append(t)
    if stopwords:
        s = set(stopwords)
        out = [t for t in out if t not in s]
    return out


@udf("tokenize_ko")
def tokenize_ko(text, mode: str | None = None, stopwords=None, stoptags=None, userdict=None):
    if text is None:
        return None
    return [t for _, t in _runs(str(text))]


@udf("stoptags_exclude")
def stoptags_exclude(tags, lang: str = "ja"):
    """Kuromoji part-of-speech tags minus the given ones (the tag inventory is not bundled:
    returns the input tags unchanged)."""
    return list(tags or [])
