"""NLP tokenizers (upstream nlp/src/main/java/hivemall/nlp/tokenizer/
{KuromojiUDF,SmartcnUDF,TokenizeKoUDF}.java, StoptagsExcludeUDF).

Upstream wraps Lucene's Kuromoji / SmartCN / Nori analyzers, which need dictionaries that are
not available offline.  These functions keep the SQL surface with a dictionary-free
segmentation: text is split into runs of one script (Han, Hiragana, Katakana, Hangul, Latin
letters/digits); Hiragana runs that follow Han are attached to it (okurigana), and Han runs in
``tokenize_cn`` are split into overlapping bigrams (the classic CJK bigram analyzer).  Output is
deterministic; tokens differ from a morphological analyzer (docs/compat.md).

Part-of-speech filtering (``stoptags``) works on a coarse tag guessed from the run's script
(Han / Katakana / Latin -> 名詞-一般, digits -> 名詞-数, Hiragana particles and auxiliaries from a
closed list -> 助詞 / 助動詞, other Hiragana -> 動詞-自立), so ``stoptags_exclude(array('名詞'))``
keeps the nouns as upstream's recipe intends.  ``stoptags_exclude`` returns the IPADIC tag
inventory Kuromoji uses minus every tag under the given ones.
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


# IPADIC part-of-speech inventory (the tag set of Kuromoji's default stoptags file), in
# hierarchy order; "-" separates the levels.
IPADIC_TAGS = (
    "その他", "その他-間投", "フィラー", "副詞", "副詞-一般", "副詞-助詞類接続", "助動詞",
    "助詞", "助詞-並立助詞", "助詞-係助詞", "助詞-副助詞", "助詞-副助詞／並立助詞／終助詞",
    "助詞-副詞化", "助詞-接続助詞", "助詞-格助詞", "助詞-格助詞-一般", "助詞-格助詞-引用",
    "助詞-格助詞-連語", "助詞-特殊", "助詞-終助詞", "助詞-連体化", "助詞-間投助詞",
    "動詞", "動詞-接尾", "動詞-自立", "動詞-非自立",
    "名詞", "名詞-サ変接続", "名詞-ナイ形容詞語幹", "名詞-一般", "名詞-代名詞", "名詞-代名詞-一般",
    "名詞-代名詞-縮約", "名詞-副詞可能", "名詞-動詞非自立的", "名詞-固有名詞", "名詞-固有名詞-一般",
    "名詞-固有名詞-人名", "名詞-固有名詞-人名-一般", "名詞-固有名詞-人名-名", "名詞-固有名詞-人名-姓",
    "名詞-固有名詞-地域", "名詞-固有名詞-地域-一般", "名詞-固有名詞-地域-国", "名詞-固有名詞-組織",
    "名詞-引用文字列", "名詞-形容動詞語幹", "名詞-接尾", "名詞-接尾-サ変接続", "名詞-接尾-一般",
    "名詞-接尾-人名", "名詞-接尾-副詞可能", "名詞-接尾-助動詞語幹", "名詞-接尾-助数詞",
    "名詞-接尾-地域", "名詞-接尾-形容動詞語幹", "名詞-接尾-特殊", "名詞-接続詞的", "名詞-数",
    "名詞-特殊", "名詞-特殊-助動詞語幹", "名詞-非自立", "名詞-非自立-一般", "名詞-非自立-副詞可能",
    "名詞-非自立-助動詞語幹", "名詞-非自立-形容動詞語幹",
    "形容詞", "形容詞-接尾", "形容詞-自立", "形容詞-非自立", "感動詞",
    "接続詞", "接頭詞", "接頭詞-形容詞接続", "接頭詞-数接続", "接頭詞-動詞接続", "接頭詞-名詞接続",
    "記号", "記号-アルファベット", "記号-一般", "記号-句点", "記号-括弧閉", "記号-括弧開",
    "記号-空白", "記号-読点", "連体詞", "非言語音", "未知語",
)

_PARTICLE = {
    "が": "助詞-格助詞-一般", "を": "助詞-格助詞-一般", "に": "助詞-格助詞-一般", "へ": "助詞-格助詞-一般",
    "で": "助詞-格助詞-一般", "から": "助詞-格助詞-一般", "より": "助詞-格助詞-一般", "と": "助詞-格助詞-一般",
    "は": "助詞-係助詞", "も": "助詞-係助詞", "こそ": "助詞-係助詞", "まで": "助詞-副助詞",
    "など": "助詞-副助詞", "だけ": "助詞-副助詞", "ばかり": "助詞-副助詞", "の": "助詞-連体化",
    "や": "助詞-並立助詞", "か": "助詞-副助詞／並立助詞／終助詞", "ね": "助詞-終助詞", "よ": "助詞-終助詞",
    "な": "助詞-終助詞", "ば": "助詞-接続助詞", "て": "助詞-接続助詞", "ので": "助詞-接続助詞",
    "けど": "助詞-接続助詞", "として": "助詞-格助詞-連語", "について": "助詞-格助詞-連語",
}
_AUX = set("た だ です ます ない ぬ れる られる せる させる う よう らしい たい".split())


def _pos(kind: str, tok: str) -> str:
    """Coarse IPADIC tag of a script run (see the module docstring)."""
    if kind == "latin":
        return "名詞-数" if tok.isdigit() else "名詞-一般"
    if kind == "hira":
        if tok in _PARTICLE:
            return _PARTICLE[tok]
        return "助動詞" if tok in _AUX else "動詞-自立"
    return "名詞-一般"


def _under(tag: str, tags) -> bool:
    """``tag`` equals one of ``tags`` or lies below it in the hierarchy."""
    return any(tag == t or tag.startswith(t + "-") for t in tags)


@udf("tokenize_ja", "tokenize_ja_neologd")
def tokenize_ja(text, mode: str | None = None, stopwords=None, stoptags=None, userdict=None):
    if text is None:
        return None
    stop = _JA_STOP if stopwords is None else set(stopwords)
    tags = list(stoptags) if stoptags else None
    return [t for kind, t in _runs(str(text))
            if t not in stop and not (tags and _under(_pos(kind, t), tags))]


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
    out = [t for _, t in _runs(str(text))]
    if stopwords:
        s = set(stopwords)
        out = [t for t in out if t not in s]
    return out


@udf("stoptags_exclude")
def stoptags_exclude(tags, lang: str = "ja"):
    """The Kuromoji (IPADIC) part-of-speech inventory minus the given tags and everything under
    them: ``stoptags_exclude(array('名詞'))`` is every non-noun tag (upstream
    StoptagsExcludeUDF; only ``lang = 'ja'`` has an inventory)."""
    if (lang or "ja").lower() != "ja":
        raise ValueError(f"stoptags_exclude: unsupported language {lang!r} (only 'ja')")
    ex = [t for t in (tags or []) if t]
    return [t for t in IPADIC_TAGS if not _under(t, ex)]
