"""Schema / feature pipeline / split / windows / CSV ingest (SURVEY.md §4 unit tier)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from wellflow.data.features import (FeaturePipeline, StringIndexer, make_windows, one_hot,
                                    random_split, take)
from wellflow.data.io import load_table, read_csv, write_csv
from wellflow.data.schema import FLOAT, INT, STRING, map_type, parse_schema
from wellflow.data.synth import TABLE_COLUMNS, TABLE_TYPES, synth_lstm_batch, well_log_table

NAMES = ",".join(TABLE_COLUMNS)
TYPES = ",".join(TABLE_TYPES)


def test_type_mapping_keeps_reference_catch_all():
    # cnn.py:55-59: only "int" and "float" are numeric; "double" becomes a string column
    assert map_type("int") == INT and map_type("float") == FLOAT
    for t in ("double", "string", "bool", "Float", ""):
        assert map_type(t) == STRING


def test_parse_schema_and_repr():
    s = parse_schema("a,b,c", "int,float,double")
    assert s.names == ["a", "b", "c"]
    assert [f.kind for f in s.fields] == [INT, FLOAT, STRING]
    assert str(s).startswith("StructType([StructField('a', IntegerType(), True)")
    assert s.categorical() == ["c"] and s.continuous() == ["a", "b"]
    assert s.continuous(exclude=("b",)) == ["a"]
    with pytest.raises(ValueError):
        parse_schema("a,b", "int")


def test_string_indexer_frequency_desc_ties_alphabetical():
    ix = StringIndexer("c").fit(["b", "a", "c", "b", "a", "d", "b"])
    assert ix.labels == ["b", "a", "c", "d"]
    assert ix.transform(["d", "b", "zz"]).tolist() == [3, 0, 4]  # unseen -> extra index
    with pytest.raises(ValueError):
        StringIndexer("c", handle_invalid="error").fit(["a"]).transform(["b"])


def test_one_hot_drop_last():
    out = one_hot(np.array([0, 1, 2]), 3, drop_last=True)
    assert out.tolist() == [[1, 0], [0, 1], [0, 0]]
    assert one_hot(np.array([2]), 3, drop_last=False).tolist() == [[0, 0, 1]]


@settings(max_examples=25, deadline=None)
@given(st.integers(50, 3000), st.integers(0, 10_000))
def test_random_split_partition_and_ratio(n, seed):
    parts = random_split(n, (0.64, 0.16, 0.2), seed)
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(n))
    assert [p.tolist() for p in parts] == [p.tolist() for p in random_split(n, (0.64, 0.16, 0.2), seed)]
    if n >= 1000:
        assert abs(len(parts[0]) / n - 0.64) < 0.06


def test_pipeline_fit_on_train_excludes_target_and_standardises():
    tbl = well_log_table(4, 50, seed=1)
    schema = parse_schema(NAMES, TYPES)
    idx = random_split(200, seed=3)
    pipe = FeaturePipeline(schema, "flow", standardize_target=True).fit(take(tbl, idx[0]))
    assert "flow" not in pipe.continuous
    X, y = pipe.transform(take(tbl, idx[0]))
    # one-hot(well: 4 labels + unknown - dropLast = 4) + one-hot(field) + 7 continuous
    assert X.shape[1] == pipe.n_features
    nc = len(pipe.continuous)
    assert np.allclose(X[:, -nc:].mean(0), 0, atol=1e-4)
    assert abs(float(y.mean())) < 1e-4
    Xv, _ = pipe.transform(take(tbl, idx[1]))  # same vocabulary on other splits
    assert Xv.shape[1] == X.shape[1]


def test_make_windows_respects_groups():
    X = np.arange(10, dtype=np.float32).reshape(10, 1)
    y = np.arange(10, dtype=np.float32)
    g = np.array([0] * 4 + [1] * 6)
    Xw, yw = make_windows(X, y, 3, g)
    assert Xw.shape == (2 + 4, 3, 1)
    assert yw.tolist() == [2, 3, 6, 7, 8, 9]
    assert Xw[2, :, 0].tolist() == [4, 5, 6]


def test_csv_roundtrip_headerless(tmp_path):
    tbl = well_log_table(2, 20, seed=0)
    p = tmp_path / "d.csv"
    write_csv(tbl, str(p), columns=TABLE_COLUMNS, header=False)
    schema = parse_schema(NAMES, TYPES)
    back = read_csv(str(p), schema)
    assert back["well"].tolist() == [str(v) for v in tbl["well"]]
    assert np.allclose(back["whp"], tbl["whp"], rtol=1e-6)
    assert back["t"].dtype == np.int64
    same = load_table(str(p), schema)
    assert len(same["flow"]) == 40


def test_csv_drops_unparseable_numeric_rows(tmp_path):
    p = tmp_path / "bad.csv"
    p.write_text("1,2.5,a\nx,3.0,b\n4,5.0,c\n")
    back = read_csv(str(p), parse_schema("i,f,s", "int,float,string"))
    assert back["i"].tolist() == [1, 4] and back["s"].tolist() == ["a", "c"]


def test_synthetic_batches_are_finite_and_learnable_scale():
    x, y = synth_lstm_batch(64, 32, 16, seed=0)
    assert x.shape == (64, 32, 16) and y.shape == (64,)
    assert np.isfinite(x.numpy()).all() and np.isfinite(y.numpy()).all()
    assert 0.2 < float(y.std()) < 3.0


def test_sequence_pipeline_fits_on_training_windows_only():
    """LSTM/CNN windows are split in time blocks; scaling statistics and vocabularies must
    come from the rows the TRAINING windows cover, not the whole file."""
    import numpy as np

    from wellflow.config import parse_argv
    from wellflow.data.features import take, time_block_split, window_rows, window_starts
    from wellflow.data.pipeline import _group_ids, _sort_by_group, prepare
    from wellflow.data.io import load_table
    from wellflow.data.schema import parse_schema

    names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
    types = "string,string,int,float,float,float,float,float,float,float"
    cfg = parse_argv("lstm", [names, types, "flow", "/tmp/x/", "--synth-wells", "4", "--synth-steps", "90",
                              "--seq-len", "16"])
    prep = prepare(cfg)
    schema = parse_schema(names, types)
    table = load_table("synth", schema, synth_wells=4, synth_steps=90, seed=cfg.seed)
    ids, _ = _group_ids(table, schema, "")
    table, ids = _sort_by_group(table, ids, schema)
    starts = window_starts(len(ids), 16, ids)
    tr, va, te = time_block_split(starts, 16, ids, cfg.split, cfg.seed)
    train_rows = window_rows(starts[tr], 16)
    assert len(train_rows) < len(ids)  # some rows are only in val/test windows
    y_train = np.asarray(take(table, train_rows)["flow"], np.float32)
    assert abs(prep.pipeline.y_mean - float(y_train.mean())) < 1e-4
    assert (len(prep.train[0]), len(prep.val[0]), len(prep.test[0])) == (len(tr), len(va), len(te))


@pytest.mark.parametrize("span", [1, 7, 16, 64])
def test_time_block_split_has_no_row_leak(span):
    """Round-1 advice: overlapping stride-1 windows split at random leak test rows into
    training. With the time-block split no row of a val/test window (inputs AND target) lies
    inside any training window, and no test row inside a val window; proportions hold."""
    import numpy as np

    from wellflow.data.features import time_block_split, window_rows, window_starts

    # 40 rows: too short to cut at every span -> assigned whole; the others are cut in time
    g = np.repeat(np.arange(5), [400, 250, 900, 600, 40])
    starts = window_starts(len(g), span, g)
    tr, va, te = time_block_split(starts, span, g)
    assert len(np.intersect1d(tr, va)) == len(np.intersect1d(tr, te)) == len(np.intersect1d(va, te)) == 0
    rows_tr, rows_va, rows_te = (set(window_rows(starts[i], span).tolist()) for i in (tr, va, te))
    assert not (rows_tr & rows_va) and not (rows_tr & rows_te) and not (rows_va & rows_te)
    n = len(tr) + len(va) + len(te)
    assert abs(len(tr) / n - 0.64) < 0.03 and abs(len(te) / n - 0.2) < 0.03
    # three short series only: each split gets one whole series
    g3 = np.repeat(np.arange(3), [30, 30, 30])
    st3 = window_starts(len(g3), 20, g3)
    parts = time_block_split(st3, 20, g3)
    assert all(len(p) for p in parts) and len(set(g3[st3[np.concatenate(parts)]])) == 3
    for k in range(5):  # time order inside every series: train < val < test
        sel = lambda ix: ix[g[starts[ix]] == k]  # noqa: E731
        a, b, c = sel(tr), sel(va), sel(te)
        if len(b) and len(c):
            assert a.max() < b.min() and b.max() < c.min()


def test_random_window_split_still_available():
    from wellflow.config import parse_argv

    names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
    types = "string,string,int,float,float,float,float,float,float,float"
    cfg = parse_argv("lstm", [names, types, "flow", "/tmp/x/", "--window-split", "random"])
    assert cfg.window_split == "random"


def test_series_windows_match_materialised_windows():
    import numpy as np
    import torch

    from wellflow.data.features import SeriesWindows, make_windows, window_starts

    rng = np.random.default_rng(0)
    X = rng.standard_normal((50, 3)).astype(np.float32)
    y = rng.standard_normal(50).astype(np.float32)
    g = np.repeat([0, 1, 2], [20, 12, 18])
    st = window_starts(50, 7, g)
    Xw, yw = make_windows(X, y, 7, g)
    sw = SeriesWindows(X, st, 7)
    assert sw.shape == Xw.shape and len(sw) == len(Xw)
    sel = np.array([5, 0, 17, 3])
    assert np.array_equal(sw[sel], Xw[sel])
    dev = sw.to("cpu")
    assert torch.equal(dev[torch.as_tensor(sel)], torch.as_tensor(Xw[sel]))
    assert np.array_equal(sw.materialize(), Xw)
