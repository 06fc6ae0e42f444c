"""NLP UDFs (hivemall_amd/nlp; upstream nlp/.../KuromojiUDF, SmartcnUDF, TokenizeKoUDF,
StoptagsExcludeUDF).  Segmentation is dictionary-free (docs/compat.md): these pin the
deterministic behaviour and the tag-inventory semantics of stoptags_exclude."""
import pandas as pd
import pytest

from hivemall_amd.nlp import IPADIC_TAGS, stoptags_exclude, tokenize_cn, tokenize_ja, tokenize_ko


def test_stoptags_exclude_drops_the_given_subtrees():
    tags = stoptags_exclude(["名詞"])
    assert tags and not any(t == "名詞" or t.startswith("名詞-") for t in tags)
    assert "助詞-格助詞-一般" in tags and "記号-句点" in tags
    assert len(tags) == len(IPADIC_TAGS) - sum(t.split("-")[0] == "名詞" for t in IPADIC_TAGS)
    # a leaf is removed alone; its parent and siblings stay
    t2 = stoptags_exclude(["助詞-格助詞-一般"])
    assert "助詞-格助詞-一般" not in t2 and "助詞-格助詞" in t2 and "助詞-格助詞-引用" in t2
    # a prefix that is not a whole level does not match ("名" is not a tag)
    assert stoptags_exclude(["名"]) == list(IPADIC_TAGS)
    assert stoptags_exclude([]) == list(IPADIC_TAGS) and len(set(IPADIC_TAGS)) == len(IPADIC_TAGS)
    with pytest.raises(ValueError):
        stoptags_exclude(["名詞"], "ko")


def test_tokenize_ja_runs_and_stoptags_keep_nouns():
    text = "東京タワーは333メートルです"
    assert tokenize_ja(text, None, []) == ["東京", "タワー", "は", "333", "メートル", "です"]
    assert tokenize_ja(text) == ["東京", "タワー", "333", "メートル", "です"]          # default stopwords drop は
    nouns = tokenize_ja(text, None, [], stoptags_exclude(["名詞"]))
    assert nouns == ["東京", "タワー", "333", "メートル"]                               # 助詞 / 助動詞 removed
    no_num = tokenize_ja(text, None, [], ["名詞-数"])
    assert "333" not in no_num and "東京" in no_num
    assert tokenize_ja(None) is None


def test_tokenize_cn_bigrams_and_ko_stopwords():
    assert tokenize_cn("我爱北京天安门") == ["我爱", "爱北", "北京", "京天", "天安", "安门"]
    assert tokenize_cn("北京 abc", ["abc"]) == ["北京"]
    assert tokenize_ko("한국어 형태소 분석", None, ["분석"]) == ["한국어", "형태소"]


def test_nlp_sql_surface():
    from hivemall_amd.sql import Session

    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"txt": ["東京タワーは333メートルです"]}))
    out = s.sql("SELECT tokenize_ja(txt, 'normal', array(), stoptags_exclude(array('名詞'))) AS w FROM t")
    assert list(out.w[0]) == ["東京", "タワー", "333", "メートル"]
