"""SQL golden tests: Hivemall's documented HiveQL patterns."""
import numpy as np
import pandas as pd
import pytest

from hivemall_amd.io.synthetic import a9a_like
from hivemall_amd.sql import Session, SQLError


@pytest.fixture
def sess():
    rows, y = a9a_like(3000)
    trows, ty = a9a_like(600, seed=4)
    s = Session(device="cpu")
    s.register("train", pd.DataFrame({"rowid": range(len(rows)),
                                      "features": [[str(int(i)) for i in r] for r in rows], "label": y}))
    s.register("test", pd.DataFrame({"rowid": range(len(trows)),
                                     "features": [[str(int(i)) for i in r] for r in trows], "label": ty}))
    return s


def test_a9a_logistic_pipeline(sess):
    sess.sql("""
    add jar hivemall-core.jar;
    source define-all.hive;
    create temporary function train_classifier as 'hivemall.classifier.GeneralClassifierUDTF';
    CREATE TABLE model AS
    SELECT feature, avg(weight) as weight FROM (
      SELECT train_classifier(add_bias(features), label, '-loss logloss -opt adagrad -reg no -iters 3')
             AS (feature, weight)
      FROM train) t GROUP BY feature;
    CREATE TABLE test_exploded AS
    SELECT rowid, label, extract_feature(fv) AS feature, extract_weight(fv) AS value
    FROM test LATERAL VIEW explode(add_bias(features)) t AS fv;
    CREATE TABLE pred AS
    SELECT t.rowid, sigmoid(sum(m.weight * t.value)) AS prob, max(t.label) AS label
    FROM test_exploded t LEFT OUTER JOIN model m ON (t.feature = m.feature)
    GROUP BY t.rowid;
    """)
    r = sess.sql("SELECT auc(prob, label) AS auc, logloss(prob, label) AS ll, count(*) AS n FROM pred")
    assert r["n"][0] == 600 and r["auc"][0] > 0.8 and r["ll"][0] < 0.6
    assert list(sess.table("model").columns) == ["feature", "weight"]


def test_arow_argmin_kld_mix(sess):
    m = sess.sql("""
    SELECT feature, argmin_kld(weight, covar) AS weight FROM (
      SELECT train_arow(add_bias(features), label) AS (feature, weight, covar) FROM train
      UNION ALL
      SELECT train_arow(add_bias(features), label, '-r 0.2') AS (feature, weight, covar) FROM train
    ) t GROUP BY feature""")
    assert len(m) >= 100 and m["weight"].notna().all()


def test_multiclass_predict_with_maxrow(sess):
    sess.sql("""
    CREATE TABLE mtrain AS SELECT rowid, features, CAST(pmod(CAST(features[0] AS int), 3) AS int) AS label FROM train;
    CREATE TABLE mmodel AS SELECT train_multiclass_scw(features, label) AS (label, feature, weight, covar) FROM mtrain;
    CREATE TABLE scores AS
    SELECT t.rowid, m.label, sum(m.weight) AS score
    FROM (SELECT rowid, fv AS feature FROM mtrain LATERAL VIEW explode(features) e AS fv) t
    JOIN mmodel m ON (t.feature = m.feature)
    GROUP BY t.rowid, m.label;
    """)
    pred = sess.sql("""
    SELECT rowid, maxrow(score, label)[1] AS predicted FROM scores GROUP BY rowid""")
    truth = sess.table("mtrain").set_index("rowid")["label"]
    acc = np.mean([truth[r] == p for r, p in zip(pred["rowid"], pred["predicted"])])
    assert acc > 0.9


def test_fm_sql_predict_matches_trainer():
    from hivemall_amd.models.fm import FMTrainer
    rng = np.random.default_rng(0)
    # index 0 is reserved for the bias (add_bias), like upstream
    rows = [[f"{int(i) + 1}:1" for i in rng.choice(100, size=5, replace=False)] for _ in range(400)]
    y = rng.random(400).astype(np.float32)
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"rowid": range(400), "features": rows, "y": y}))
    s.sql("CREATE TABLE fm_model AS SELECT train_fm(features, y, '-factors 3 -iters 2') AS (feature, Wi, Vif) FROM t")
    p = s.sql("""
    SELECT t.rowid, fm_predict(m.Wi, m.Vif, t.Xi) AS p FROM (
      SELECT rowid, extract_feature(fv) AS feature, extract_weight(fv) AS Xi
      FROM t LATERAL VIEW explode(add_bias(features)) e AS fv) t
    LEFT OUTER JOIN fm_model m ON (t.feature = m.feature)
    GROUP BY t.rowid ORDER BY rowid""")
    tr = FMTrainer("-factors 3 -iters 2", device="cpu").fit(rows, y)
    ref = tr.predict(rows)
    np.testing.assert_allclose(p["p"].to_numpy(dtype=float), ref, rtol=1e-3, atol=1e-4)


def test_ffm_sql_predict_matches_trainer():
    from hivemall_amd.models.ffm import FFMTrainer
    rng = np.random.default_rng(1)
    rows = [[f"{f}:{int(rng.integers(0, 20))}:1" for f in range(4)] for _ in range(300)]
    y = (rng.random(300) < 0.4).astype(int)
    opts = "-c -factors 2 -num_fields 4 -feature_hashing 10 -iters 2 -w0"
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"rowid": range(300), "features": rows, "label": y}))
    s.sql(f"CREATE TABLE ffm_model AS SELECT train_ffm(features, label, '{opts}') AS (model_id, i, Wi, Vi) FROM t")
    p = s.sql("""
    SELECT t.rowid, sigmoid(ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj)) AS p FROM (
      SELECT rowid, i, j, Xi, Xj FROM t
      LATERAL VIEW feature_pairs(features, '-ffm -feature_hashing 10 -num_fields 4') x AS i, j, Xi, Xj) t
    LEFT OUTER JOIN ffm_model m1 ON (t.i = m1.i)
    LEFT OUTER JOIN ffm_model m2 ON (t.j = m2.i)
    GROUP BY t.rowid ORDER BY rowid""")
    tr = FFMTrainer(opts, device="cpu").fit(rows, y)
    ref = tr.predict(rows)
    np.testing.assert_allclose(p["p"].to_numpy(dtype=float), ref, rtol=1e-4, atol=1e-5)


def test_query_features():
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"g": ["a", "a", "b", "b", "b"], "x": [1, 2, 3, 4, 5]}))
    r = s.sql("""
    WITH w AS (SELECT g, x, row_number() OVER (PARTITION BY g ORDER BY x DESC) AS rn FROM t)
    SELECT g, x FROM w WHERE rn = 1 ORDER BY g""")
    assert r.values.tolist() == [["a", 2], ["b", 5]]
    r = s.sql("SELECT g, sum(x) s, count(*) c FROM t GROUP BY g HAVING sum(x) > 5 ORDER BY s DESC")
    assert r.values.tolist() == [["b", 12, 3]]
    r = s.sql("SELECT CASE WHEN x > 2 THEN 'hi' ELSE 'lo' END AS k, x BETWEEN 2 AND 4 AS b, "
              "x IN (1, 5) AS i FROM t ORDER BY x")
    assert r["k"].tolist() == ["lo", "lo", "hi", "hi", "hi"]
    assert r["b"].tolist() == [False, True, True, True, False]
    s.sql("CREATE TEMPORARY MACRO max3(a, b, c) max2(max2(a, b), c)")
    assert s.sql("SELECT max3(1, 7, 3) AS m")["m"][0] == 7
    s.sql("set hivevar:lim=2")
    assert len(s.sql("SELECT * FROM t LIMIT ${lim}")) == 2
    r = s.sql("SELECT x FROM t WHERE g = 'a' UNION ALL SELECT x FROM t WHERE x > 4")
    assert sorted(r["x"].tolist()) == [1, 2, 5]
    r = s.sql("SELECT each_top_k(2, g, x, g, x) AS (rank, key, gg, xx) FROM (SELECT * FROM t CLUSTER BY g) t")
    assert len(r) == 4
    with pytest.raises(SQLError):
        s.sql("SELECT nope FROM t")
    assert "train_ffm" in s.sql("SHOW FUNCTIONS")["tab_name"].tolist()


def test_amplify_and_rand_amplify(sess):
    r = sess.sql("SELECT amplify(3, rowid, label) AS (rowid, label) FROM train")
    assert len(r) == 9000
    r = sess.sql("SELECT rand_amplify(2, 100, rowid, label) AS (rowid, label) FROM train")
    assert len(r) == 6000 and sorted(r["rowid"].tolist()) == sorted(list(range(3000)) * 2)


@pytest.mark.parametrize("opt", ["-ffm -feature_hashing 10 -num_fields 7", "-ffm -feature_hashing 10 -num_fields 7 -no_bias"])
def test_feature_pairs_batch_path_equals_per_row(opt, monkeypatch):
    """LATERAL VIEW feature_pairs('-ffm'): the column-at-once path (models/ffm_keys.
    ffm_pair_columns) returns the per-row generator's table exactly — rows, order, dtypes,
    NULLs — including NULL rows, empty rows, named features and explicit values."""
    rng = np.random.default_rng(3)
    rows = []
    for _ in range(400):
        nf = int(rng.integers(0, 7))
        rows.append([f"{f}:{int(rng.integers(0, 30))}" + (f":{rng.uniform(0.1, 3):.3f}" if rng.random() < 0.5 else "")
                     for f in range(nf)])
    rows[3] = None
    rows[5] = ["2:abc:1.5", "0:xyz"]
    df = pd.DataFrame({"rowid": range(400), "features": rows})
    q = f"SELECT rowid, i, j, Xi, Xj FROM t LATERAL VIEW feature_pairs(features, '{opt}') x AS i, j, Xi, Xj"
    out = []
    for mode in ("1", "0"):
        monkeypatch.setenv("HM_SQL_BATCH_UDTF", mode)
        s = Session(device="cpu")
        s.register("t", df)
        out.append(s.sql(q))
    pd.testing.assert_frame_equal(out[0], out[1])


def test_file_backed_tables_and_cli(tmp_path):
    """CREATE EXTERNAL TABLE ... LOCATION (libsvm, delimited text with arrays, parquet), LOAD
    DATA INPATH, INSERT OVERWRITE LOCAL DIRECTORY and the `python -m hivemall_amd.sql` runner
    (io/tables.py)."""
    import pandas as pd
    import pyarrow as pa
    import pyarrow.parquet as pq

    from hivemall_amd.sql import Session
    from hivemall_amd.sql.__main__ import main as cli

    (tmp_path / "a9a.libsvm").write_text("1 3:1 5:0.5 7:1\n-1 2:1 5:1\n\n1 1:0.25 3:1 9:1\n")
    (tmp_path / "t.tsv").write_text("1\tapple,banana\t0.5\n0\tcherry\t\\N\n")
    pq.write_table(pa.table({"rowid": [1, 2], "features": [["1:0.5", "2:1"], ["3:1"]]}),
                   tmp_path / "test.parquet")
    s = Session(device="cpu")
    s.sql(f"""
        CREATE EXTERNAL TABLE a9a (label double, features array<string>) STORED AS libsvm
          LOCATION '{tmp_path}/a9a.libsvm';
        CREATE TABLE t (id int, tags array<string>, w double)
          ROW FORMAT DELIMITED FIELDS TERMINATED BY '\\t' COLLECTION ITEMS TERMINATED BY ','
          STORED AS TEXTFILE;
        LOAD DATA LOCAL INPATH '{tmp_path}/t.tsv' OVERWRITE INTO TABLE t;
        CREATE EXTERNAL TABLE test (rowid bigint, features array<string>) STORED AS PARQUET
          LOCATION '{tmp_path}/test.parquet';
    """)
    a9a = s.table("a9a")
    assert a9a["label"].tolist() == [1.0, -1.0, 1.0]
    assert [list(f) for f in a9a["features"]] == [["3:1", "5:0.5", "7:1"], ["2:1", "5:1"], ["1:0.25", "3:1", "9:1"]]
    t = s.table("t")
    assert t["id"].tolist() == [1, 0] and [list(x) for x in t["tags"]] == [["apple", "banana"], ["cherry"]]
    assert t["w"].iloc[0] == 0.5 and pd.isna(t["w"].iloc[1])
    assert isinstance(s.table("test")["features"].dtype, pd.ArrowDtype)
    m = s.sql("SELECT train_classifier(add_bias(features), label, '-loss logloss') AS (feature, weight) FROM a9a")
    assert sorted(m["feature"].tolist()) == ["0", "1", "2", "3", "5", "7", "9"]
    # INSERT OVERWRITE DIRECTORY writes Hive text; reading it back with the same declaration
    s.sql(f"INSERT OVERWRITE LOCAL DIRECTORY '{tmp_path}/out' ROW FORMAT DELIMITED FIELDS TERMINATED BY '\\t' "
          "COLLECTION ITEMS TERMINATED BY ',' SELECT id, tags, w FROM t")
    assert (tmp_path / "out" / "000000_0").read_text() == "1\tapple,banana\t0.5\n0\tcherry\t\\N\n"
    s.sql(f"CREATE EXTERNAL TABLE t2 (id int, tags array<string>, w double) ROW FORMAT DELIMITED "
          f"FIELDS TERMINATED BY '\\t' COLLECTION ITEMS TERMINATED BY ',' LOCATION '{tmp_path}/out'")
    t2 = s.table("t2")
    assert t2["id"].tolist() == t["id"].tolist() and [list(x) for x in t2["tags"]] == [list(x) for x in t["tags"]]
    # the command-line runner: a registered file, a script with ${hivevar:...}, --out
    (tmp_path / "q.sql").write_text("SELECT label, size(features) AS n FROM ${hivevar:tab} WHERE label > 0;")
    assert cli(["-f", str(tmp_path / "q.sql"), "--device", "cpu", "--hivevar", "tab=x",
                "--table", f"x={tmp_path}/a9a.libsvm", "--out", str(tmp_path / "r.tsv")]) == 0
    assert (tmp_path / "r.tsv").read_text() == "1.0\t3\n1.0\t3\n"


def test_lexer_octal_and_unicode_escapes():
    from hivemall_amd.sql.lexer import tokenize

    vals = [t.val for t in tokenize(r"select '\001', '\t', '\u0002', 'a\nb', '\0'") if t.kind == "str"]
    assert vals == ["\x01", "\t", "\x02", "a\nb", "\x00"]


def test_udf_null_first_argument_yields_null():
    """Hivemall's NULL rule: a per-row UDF whose principal (first) argument is NULL returns
    NULL instead of raising (lat2tiley, popcnt, distance2similarity, ... on NULL rows)."""
    import pandas as pd

    from hivemall_amd.sql import Session

    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"a": [1.5, None], "b": [[1, 2], None]}, dtype=object))
    r = s.sql("SELECT popcnt(b) AS p, lat2tiley(a, 3) AS y, vectorize_features(array('x'), a) AS v FROM t")
    assert pd.isna(r["p"].iloc[1]) and pd.isna(r["y"].iloc[1]) and r["p"].iloc[0] == 2
    r2 = s.sql("SELECT distance2similarity(a) AS d FROM t")
    assert pd.isna(r2["d"].iloc[1]) and r2["d"].iloc[0] > 0


def test_show_tables_describe_and_stdin_runner(monkeypatch, capsys):
    import io

    import pandas as pd

    from hivemall_amd.sql import Session
    from hivemall_amd.sql.__main__ import main as cli

    s = Session(device="cpu")
    s.register("train", pd.DataFrame({"rowid": [1, 2], "features": [["a:1"], ["b:2"]], "label": [1.0, 0.0]}))
    s.sql("CREATE TABLE t2 (k string, v array<double>); CREATE VIEW v AS SELECT rowid FROM train")
    assert s.sql("SHOW TABLES")["tab_name"].tolist() == ["t2", "train", "v"]
    assert s.sql("SHOW TABLES 'tr*'")["tab_name"].tolist() == ["train"]
    d = s.sql("DESCRIBE train")
    assert d["data_type"].tolist() == ["bigint", "array<string>", "double"]
    assert s.sql("DESCRIBE t2")["data_type"].tolist() == ["string", "array<double>"]
    monkeypatch.setattr("sys.stdin", io.StringIO("SELECT 40 + 2 AS answer;"))
    assert cli(["--device", "cpu"]) == 0
    assert "42" in capsys.readouterr().out


def test_create_temporary_function_aliases():
    """CREATE TEMPORARY FUNCTION name AS '<class>' makes `name` callable: a Hivemall class (by its
    simple name) or one of this engine's implementations (as define-all.hive names them)."""
    import pandas as pd

    from hivemall_amd.sql import Session

    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"f": [["a:1", "b:2"]], "y": [1]}))
    s.sql("CREATE TEMPORARY FUNCTION my_hash AS 'hivemall.ftvec.hashing.FeatureHashingUDF';"
          "CREATE TEMPORARY FUNCTION my_train AS 'hivemall.classifier.GeneralClassifierUDTF';"
          "CREATE TEMPORARY FUNCTION sig AS 'hivemall_amd.tools.functions.sigmoid';"
          "CREATE TEMPORARY FUNCTION nope AS 'com.example.Missing'")
    r = s.sql("SELECT my_hash(f) AS h, sig(0) AS p FROM t")
    assert list(r["h"].iloc[0]) == list(s.sql("SELECT feature_hashing(f) AS h FROM t")["h"].iloc[0])
    assert r["p"].iloc[0] == 0.5
    m = s.sql("SELECT my_train(add_bias(f), y) AS (feature, weight) FROM t")
    assert sorted(m["feature"]) == ["0", "a", "b"]
    import pytest

    from hivemall_amd.sql import SQLError
    with pytest.raises(SQLError):
        s.sql("SELECT nope(1) FROM t")


def test_hive_date_functions_and_constructors():
    """Hive's date built-ins (UTC), zero-argument constructors broadcast to every row, and
    ``map(...)[key]`` (Hive's map constructor, not a metric alias)."""
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"rowid": [1, 2], "d": ["2020-01-02 10:11:12", "bad"]}))
    r = s.sql("SELECT from_unixtime(0) a, from_unixtime(86400, 'yyyy/MM/dd') b, "
              "unix_timestamp('1970-01-01 00:00:01') c, unix_timestamp('01/02/1970', 'MM/dd/yyyy') e, "
              "to_date(d) f, datediff('2020-01-03', '2020-01-01') g, date_add('2020-02-28', 2) h, "
              "date_sub('2020-03-01', 1) i, year(d) y, hour(d) hh, date_format(d, 'yyyy-MM') m FROM t")
    row = r.iloc[0].to_dict()
    assert row == {"a": "1970-01-01 00:00:00", "b": "1970/01/02", "c": 1, "e": 86400, "f": "2020-01-02",
                   "g": 2, "h": "2020-03-01", "i": "2020-02-29", "y": 2020, "hh": 10, "m": "2020-01"}
    assert r["f"].iloc[1] is None and r["y"].iloc[1] is None        # unparsable -> NULL
    r = s.sql("SELECT map('a', 1)['a'] a, size(array()) z FROM t")
    assert r["a"].tolist() == [1, 1] and r["z"].tolist() == [0, 0]
    r = s.sql("SELECT rowid, f FROM t LATERAL VIEW OUTER explode(array()) e AS f")
    assert r["rowid"].tolist() == [1, 2] and r["f"].isna().all()


def test_star_arguments_and_table_ddl():
    """The a9a tutorial's statements: ``amplify(3, *)``, CREATE OR REPLACE VIEW, TRUNCATE,
    ALTER TABLE ... RENAME TO, and the storage-only statements accepted as no-ops."""
    s = Session(device="cpu")
    s.register("train", pd.DataFrame({"rowid": [1, 2], "features": [["a:1"], ["b:2"]], "label": [1, 0]}))
    s.sql("CREATE TABLE x3 AS SELECT amplify(3, *) AS (rowid, features, label) FROM train")
    r = s.sql("SELECT rowid, count(*) c FROM x3 GROUP BY rowid ORDER BY rowid")
    assert r["c"].tolist() == [3, 3]
    r = s.sql("SELECT concat_ws('|', t.*) j FROM (SELECT cast(rowid AS string) a, 'z' b FROM train) t")
    assert r["j"].tolist() == ["1|z", "2|z"]
    s.sql("CREATE OR REPLACE VIEW v AS SELECT rowid FROM train WHERE label = 1")
    s.sql("CREATE OR REPLACE VIEW v AS SELECT rowid FROM train")
    assert len(s.sql("SELECT * FROM v")) == 2
    s.sql("ALTER TABLE x3 RENAME TO x3b")
    s.sql("TRUNCATE TABLE x3b")
    assert len(s.sql("SELECT * FROM x3b")) == 0 and list(s.table("x3b").columns) == ["rowid", "features", "label"]
    with pytest.raises(Exception):
        s.sql("SELECT * FROM x3")
    for q in ("CREATE DATABASE IF NOT EXISTS d", "ANALYZE TABLE x3b COMPUTE STATISTICS",
              "ALTER TABLE x3b SET TBLPROPERTIES ('a'='b')", "MSCK REPAIR TABLE x3b"):
        assert s.sql(q) is None


def test_window_frames_follow_hive_defaults():
    """ORDER BY without a frame = RANGE UNBOUNDED PRECEDING .. CURRENT ROW (peers included),
    no ORDER BY = whole partition, explicit ROWS / RANGE frames, percent_rank / cume_dist."""
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"g": ["a", "a", "a", "b", "b"], "x": [1, 2, 3, 4, 5], "y": [3, 1, 2, 1, 1]}))
    r = s.sql("SELECT sum(x) OVER (PARTITION BY g ORDER BY x) cs, sum(x) OVER (PARTITION BY g) ts, "
              "sum(x) OVER (ORDER BY y) rs, "
              "avg(x) OVER (PARTITION BY g ORDER BY x ROWS BETWEEN 1 PRECEDING AND 1 FOLLOWING) ma, "
              "last_value(x) OVER (PARTITION BY g ORDER BY x) l, "
              "count(*) OVER (ORDER BY y RANGE BETWEEN 1 PRECEDING AND CURRENT ROW) rc, "
              "sum(x) OVER (ORDER BY x ROWS 1 PRECEDING) r1, "
              "percent_rank() OVER (ORDER BY y) p, cume_dist() OVER (ORDER BY y) c FROM t")
    assert r["cs"].tolist() == [1, 3, 6, 4, 9] and r["ts"].tolist() == [6, 6, 6, 9, 9]
    assert r["rs"].tolist() == [15, 11, 14, 11, 11]
    assert r["ma"].tolist() == [1.5, 2.0, 2.5, 4.5, 4.5] and r["l"].tolist() == [1, 2, 3, 4, 5]
    assert r["rc"].tolist() == [2, 3, 4, 3, 3] and r["r1"].tolist() == [1, 3, 5, 7, 9]
    assert r["p"].tolist() == [1.0, 0.0, 0.75, 0.0, 0.0] and r["c"].tolist() == [1.0, 0.6, 0.8, 0.6, 0.6]


def test_exists_subqueries():
    """[NOT] EXISTS: uncorrelated, and correlated through equality conjuncts (a semi-join)."""
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"g": ["a", "a", "b", "c"], "x": [1, 2, 3, 4]}))
    s.register("u", pd.DataFrame({"g": ["a", "c", "c"], "y": [10, 5, 50]}))
    q = "SELECT x FROM t WHERE {} ORDER BY x"
    assert s.sql(q.format("EXISTS (SELECT 1 FROM u WHERE u.g = t.g)"))["x"].tolist() == [1, 2, 4]
    assert s.sql(q.format("NOT EXISTS (SELECT 1 FROM u WHERE u.g = t.g AND u.y > 20)"))["x"].tolist() == [1, 2, 3]
    assert s.sql(q.format("EXISTS (SELECT 1 FROM u WHERE y > 40)"))["x"].tolist() == [1, 2, 3, 4]
    assert len(s.sql(q.format("EXISTS (SELECT 1 FROM u WHERE y > 400)"))) == 0
    with pytest.raises(Exception):
        s.sql(q.format("EXISTS (SELECT 1 FROM u WHERE u.y > t.x)"))


def test_rollup_cube_grouping_sets():
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"g": ["a", "a", "b", "b"], "h": ["x", "y", "x", "x"], "v": [1, 2, 3, 4]}))
    r = s.sql("SELECT g, h, sum(v) s FROM t GROUP BY g, h WITH ROLLUP")
    assert r["s"].tolist() == [1, 2, 7, 3, 7, 10] and r["h"].isna().tolist()[3:] == [True] * 3
    r = s.sql("SELECT g, h, count(*) c FROM t GROUP BY g, h WITH CUBE")
    assert len(r) == 8 and r["c"].iloc[-1] == 4 and r["c"].sum() == 16
    r = s.sql("SELECT g, sum(v) s FROM t GROUP BY g, h GROUPING SETS ((g, h), g, ()) ORDER BY s DESC LIMIT 2")
    assert r["s"].tolist() == [10, 7] and pd.isna(r["g"].iloc[0])


def test_tablesample_and_hive_hash():
    """TABLESAMPLE(BUCKET x OUT OF y ON e | n PERCENT | n ROWS) and Hive's deterministic
    hash() (Java hash codes: ints themselves, strings the 31-polynomial of their bytes)."""
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"id": range(10), "k": list("abcdeabcde")}))
    assert s.sql("SELECT id FROM t TABLESAMPLE(BUCKET 1 OUT OF 2 ON id) s")["id"].tolist() == [0, 2, 4, 6, 8]
    assert s.sql("SELECT id FROM t TABLESAMPLE(30 PERCENT)")["id"].tolist() == [0, 1, 2]
    assert s.sql("SELECT id FROM t TABLESAMPLE(2 ROWS) x")["id"].tolist() == [0, 1]
    parts = [set(s.sql(f"SELECT id FROM t TABLESAMPLE(BUCKET {b} OUT OF 3 ON k)")["id"]) for b in (1, 2, 3)]
    assert set().union(*parts) == set(range(10)) and sum(map(len, parts)) == 10
    r = s.sql("SELECT hash('hello') a, hash(1, 'a') b, hash(cast(1.5 AS double)) c FROM t LIMIT 1")
    assert r.iloc[0].tolist() == [99162322, 128, 1073217536]


def test_more_hive_builtins():
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"x": [1.0, 2.0, 3.0, 10.0], "y": [2.0, 4.1, 6.0, 20.5], "d": ["2020-01-31"] * 4}))
    r = s.sql("SELECT conv('ff', 16, 10) a, conv('-1', 10, 16) b, hex('ab') c, unbase64(base64('hi')) e, "
              "translate('hello', 'el', 'ip') f, levenshtein('kitten', 'sitting') g, soundex('Robert') h, "
              "find_in_set('b', 'a,b,c') i, str_to_map('a:1,b:2')['b'] j, "
              "parse_url('http://h.com/p?q=1&r=2', 'QUERY', 'r') k, printf('%s-%03d', 'x', 7) l, "
              "crc32('abc') m, add_months(d, 1) n, last_day('2020-02-10') o, next_day('2020-01-01', 'MO') p, "
              "trunc('2020-05-17', 'MM') q FROM t LIMIT 1").iloc[0].to_dict()
    assert r == {"a": "255", "b": "FFFFFFFFFFFFFFFF", "c": "6162", "e": "hi", "f": "hippo", "g": 3, "h": "R163",
                 "i": 2, "j": "2", "k": "2", "l": "x-007", "m": 891568578, "n": "2020-02-29", "o": "2020-02-29",
                 "p": "2020-01-06", "q": "2020-05-01"}
    r = s.sql("SELECT covar_pop(x, y) a, covar_samp(x, y) b, histogram_numeric(x, 2) h FROM t").iloc[0]
    assert abs(r["a"] - 25.7) < 1e-9 and abs(r["b"] - 34.2666666667) < 1e-6
    assert r["h"] == [{"x": 2.0, "y": 3.0}, {"x": 10.0, "y": 1.0}]
    r = s.sql("SELECT p.host, p.path FROM t LATERAL VIEW parse_url_tuple('http://h.com/p?q=1', 'HOST', 'PATH') p "
              "AS host, path LIMIT 1")
    assert r.iloc[0].tolist() == ["h.com", "/p"]


def test_rowid_and_rownum_sequences():
    """rowid() and rownum() keep separate sequences (separate UDF instances in Hive);
    rownum() = sequence followed by the 4-digit task id."""
    from hivemall_amd.tools.functions import CONTEXT

    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"x": [1, 2, 3]}))
    r0, n0 = CONTEXT.row, CONTEXT.rownum
    r = s.sql("SELECT rowid() a, rownum() b FROM t")
    assert r["a"].tolist() == [f"{CONTEXT.task_id}-{r0 + i}" for i in (1, 2, 3)]
    assert r["b"].tolist() == [int(f"{n0 + i}{CONTEXT.task_id:04d}") for i in (1, 2, 3)]


def test_from_first_multi_insert():
    """Hive's ``FROM src INSERT ... SELECT ... INSERT ... SELECT ...`` and ``FROM src SELECT``."""
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"x": [1, 2, 3, 4], "g": ["a", "b", "a", "b"]}))
    s.sql("CREATE TABLE big (x int)")
    s.sql("FROM t INSERT OVERWRITE TABLE small SELECT x WHERE x < 3 "
          "INSERT INTO TABLE big SELECT x WHERE x >= 3 INSERT OVERWRITE TABLE agg SELECT g, sum(x) s GROUP BY g")
    assert s.table("small")["x"].tolist() == [1, 2] and s.table("big")["x"].tolist() == [3, 4]
    assert sorted(s.table("agg").itertuples(index=False, name=None)) == [("a", 4), ("b", 6)]
    assert s.sql("FROM t SELECT max(x) m")["m"].tolist() == [4]


def test_integer_div_and_mod_truncate_toward_zero():
    s = Session(device="cpu")
    r = s.sql("SELECT -7 div 2 a, 7 div 2 b, -7 % 3 c, 7 % -3 d").iloc[0].tolist()
    assert r == [-3, 3, -1, 1]


def test_create_table_like():
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"x": [1, 2], "f": [["a"], ["b"]]}))
    s.sql("CREATE TABLE u LIKE t")
    assert list(s.table("u").columns) == ["x", "f"] and len(s.table("u")) == 0
    s.sql("INSERT INTO TABLE u SELECT * FROM t WHERE x = 2")
    assert s.table("u")["x"].tolist() == [2]


def test_limit_with_offset():
    s = Session(device="cpu")
    s.register("t", pd.DataFrame({"x": range(10)}))
    assert s.sql("SELECT x FROM t ORDER BY x LIMIT 3, 2")["x"].tolist() == [3, 4]
    assert s.sql("SELECT x FROM t ORDER BY x LIMIT 2")["x"].tolist() == [0, 1]
    assert s.sql("SELECT x FROM t UNION ALL SELECT x FROM t ORDER BY x LIMIT 1, 2")["x"].tolist() == [0, 1]


def test_insert_overwrite_directory_replaces_old_data(tmp_path):
    """INSERT OVERWRITE DIRECTORY replaces the directory's data files (Hive): a stale parquet
    file from an earlier write is not read back next to the new text output."""
    import pandas as pd

    from hivemall_amd.io.tables import read_table, write_table

    d = str(tmp_path / "out")
    write_table(pd.DataFrame({"a": [1, 2, 3]}), d, "parquet", overwrite_dir=True)
    (tmp_path / "out" / "_SUCCESS").write_text("")
    write_table(pd.DataFrame({"a": [7]}), d, "textfile", overwrite_dir=True)
    import os

    assert sorted(os.listdir(d)) == ["000000_0", "_SUCCESS"]
    assert read_table(d, "textfile", ["a"], ["int"])["a"].tolist() == [7]


def _criteo_strings(n, seed=1):
    import numpy as np
    import pandas as pd
    import pyarrow as pa

    from hivemall_amd.io.synthetic import criteo_like

    idx, y = criteo_like(n, 16, seed=seed)
    names = np.char.add(np.char.add(np.arange(39).astype(str)[None, :].repeat(n, 0), "#"), idx.numpy().astype(str))
    names = names.astype(object)
    names[::7, 3] = names[::7, 3] + ":0.25"          # some explicit values
    flat = pa.array(names.reshape(-1), type=pa.string())
    col = pa.ListArray.from_arrays(pa.array(np.arange(0, n * 39 + 1, 39, dtype=np.int32)), flat)
    return pd.DataFrame({"features": pd.Series(pd.arrays.ArrowExtensionArray(col)),
                         "label": (y.numpy() > 0).astype(np.int32)})


def test_device_ftvec_matches_string_path_cpu():
    """hashed_csr_device (the GPU planner's feature_hashing + add_bias; on the CPU every chunk
    takes its host path) gives the CSR the learner's int encoder reads from the hashed strings;
    the planner matches only [add_bias(]feature_hashing(col[, const])[)]; take_rows shards."""
    import numpy as np
    import torch

    from hivemall_amd.ftvec.functions import add_bias, feature_hashing
    from hivemall_amd.io.ingest import hashed_csr_device
    from hivemall_amd.sql.device_ftvec import _match
    from hivemall_amd.sql.parser import parse_expr
    from hivemall_amd.utils.features import FeatureEncoder

    df = _criteo_strings(300)
    ref = FeatureEncoder("int").encode(add_bias(feature_hashing(df["features"], "-num_features 65536")))
    got = hashed_csr_device(df["features"], 65536, True, device="cpu", chunk_rows=128)
    assert np.array_equal(got.indptr.numpy(), ref.indptr)
    assert np.array_equal(got.idx.numpy(), ref.idx.astype(np.int64))
    assert np.array_equal(got.val.numpy(), ref.val.astype(np.float32))
    sh = got.take_rows(1, 3)
    ref1 = FeatureEncoder("int").encode(add_bias(feature_hashing(df["features"].iloc[1::3].reset_index(drop=True),
                                                                 "-num_features 65536")))
    assert np.array_equal(sh.idx.numpy(), ref1.idx) and torch.equal(sh.indptr, torch.from_numpy(ref1.indptr))

    m = _match(parse_expr("add_bias(feature_hashing(features, '-num_features 1024'))"))
    assert m is not None and m[1] == 1024 and m[2] is True
    assert _match(parse_expr("feature_hashing(features)"))[1:] == (1 << 24, False)
    assert _match(parse_expr("feature_hashing(add_bias(features))")) is None
    assert _match(parse_expr("add_bias(features)")) is None


@pytest.mark.gpu
def test_device_ftvec_sql_model_table_bit_identical(monkeypatch):
    """train_classifier(add_bias(feature_hashing(features)), ...) on a GPU session: the fused
    device path (strings hashed by hm_feat_parse into device CSR) and the string path give the
    same model table, bit for bit."""
    import numpy as np

    from hivemall_amd.sql import Session

    df = _criteo_strings(20000)
    q = ("SELECT train_classifier(add_bias(feature_hashing(features, '-num_features 262144')), label, "
         "'-loss logloss -opt adagrad -dims 262144') AS (feature, weight) FROM criteo")
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("HM_SQL_DEVICE_FTVEC", flag)
        s = Session(device="cuda")
        s.register("criteo", df)
        out[flag] = s.sql(q).sort_values("feature").reset_index(drop=True)
    a, b = out["1"], out["0"]
    assert len(a) == len(b) > 1000
    assert np.array_equal(a["feature"].to_numpy(), b["feature"].to_numpy())
    assert np.array_equal(a["weight"].to_numpy(), b["weight"].to_numpy())
