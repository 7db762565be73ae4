"""Native host runtime (csrc/runtime/, wellflow/_runtime.so): CSV ingest against the Arrow
oracle, window enumeration / gather against numpy, the background prefetcher, and the C++
self-test under ThreadSanitizer and AddressSanitizer+UBSan (host-side race / memory
checking)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from wellflow.data import native
from wellflow.data.features import window_starts_py
from wellflow.data.io import read_csv_arrow, write_csv
from wellflow.data.schema import parse_schema
from wellflow.data.synth import TABLE_COLUMNS, TABLE_TYPES, well_log_table

pytestmark = pytest.mark.skipif(not native.available(), reason="native runtime not built")

RT_DIR = os.path.join(os.path.dirname(native.__file__), "..", "csrc", "runtime")


def _same_table(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert x.shape == y.shape, k
        if x.dtype == object:
            assert list(x) == list(y), k
        else:
            np.testing.assert_array_equal(x, y, err_msg=k)


def test_csv_matches_arrow_on_well_logs(tmp_path):
    table = well_log_table(8, 300, seed=3)
    path = str(tmp_path / "logs.csv")
    write_csv(table, path, columns=TABLE_COLUMNS)
    schema = parse_schema(",".join(TABLE_COLUMNS), ",".join(TABLE_TYPES))
    _same_table(native.read_csv(path, schema), read_csv_arrow(path, schema))
    assert native.read_csv.last_dropped == 0


def test_csv_bad_rows_quotes_crlf_and_threads(tmp_path):
    lines = ['"w,1",3,1.5', "w2,4.0,2.5", "w3,x,1.0", "w4,5", "w5,6,", '"say ""hi""",7,3.25', "", "w6,8,1e2"]
    path = str(tmp_path / "bad.csv")
    with open(path, "w", newline="") as f:
        f.write("\r\n".join(lines) + "\r\n")
    schema = parse_schema("well,n,v", "string,int,float")
    got = native.read_csv(path, schema)
    assert list(got["well"]) == ["w,1", "w2", 'say "hi"', "w6"]
    np.testing.assert_array_equal(got["n"], [3, 4, 7, 8])
    np.testing.assert_allclose(got["v"], [1.5, 2.5, 3.25, 100.0])
    assert native.read_csv.last_dropped == 3  # non-integer int cell, short row, empty float
    # large file: many workers, same answer as one
    big = str(tmp_path / "big.csv")
    rng = np.random.default_rng(0)
    n = 200_000
    with open(big, "w") as f:
        for i in range(n):
            f.write(f"s{rng.integers(0, 50)},{i},{i * 0.25}\n")
    a = native.read_csv(big, schema, threads=1)
    b = native.read_csv(big, schema, threads=8)
    _same_table(a, b)
    np.testing.assert_array_equal(a["n"], np.arange(n))


def test_window_starts_and_gather_match_numpy():
    rng = np.random.default_rng(1)
    groups = np.repeat(np.arange(7), rng.integers(1, 40, size=7))
    n, T = len(groups), 6
    for stride in (1, 3):
        np.testing.assert_array_equal(native.window_starts(n, T, groups, stride), window_starts_py(n, T, groups, stride))
    np.testing.assert_array_equal(native.window_starts(n, T, None), window_starts_py(n, T, None))
    starts = window_starts_py(n, T, groups)
    rows = rng.standard_normal((n, 5)).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    idx = rng.permutation(len(starts))[:37]
    xw, yw = native.gather_windows(rows, starts, T, idx=idx, y=y)
    ref = rows[starts[idx][:, None] + np.arange(T)[None, :]]
    np.testing.assert_array_equal(xw, ref)
    np.testing.assert_array_equal(yw, y[starts[idx] + T - 1])


def test_prefetcher_ring():
    rng = np.random.default_rng(2)
    n, T, F, B = 500, 8, 4, 32
    rows = rng.standard_normal((n, F)).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    starts = window_starts_py(n, T)
    pf = native.Prefetcher(rows, starts, y, T, B, nslots=3, threads=3)
    batches = [rng.integers(0, len(starts), size=B) for _ in range(9)]
    for k in range(3):
        pf.submit(k, batches[k])
    for k in range(9):
        x, yy = pf.wait(k % 3)
        st = starts[batches[k]]
        np.testing.assert_array_equal(x.numpy(), rows[st[:, None] + np.arange(T)[None, :]])
        np.testing.assert_array_equal(yy.numpy(), y[st + T - 1])
        if k + 3 < 9:
            pf.submit(k % 3, batches[k + 3])
    pf.close()


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_native_selftest_under_sanitizers(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    exe = str(tmp_path / "selftest")
    srcs = [os.path.join(RT_DIR, f) for f in ("selftest.cpp", "csv.cpp", "windows.cpp")]
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer",
                    f"-I{RT_DIR}", *srcs, "-o", exe], check=True, capture_output=True)
    r = subprocess.run([exe, str(tmp_path / "st.csv")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "selftest ok" in r.stdout, r.stdout + r.stderr
