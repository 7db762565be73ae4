"""tools/mfma_war.py: the static check for instructions that touch an inline-asm MFMA's
operands right after issue (the hazard class behind the round-2 forward bug)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("mfma_war", os.path.join(ROOT, "tools", "mfma_war.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ASM = """
_Z4kernv:
\tv_mfma_f32_16x16x32_bf16 a[24:27], v[12:15], a[84:87], a[24:27]
\ts_nop 0
\tv_accvgpr_read_b32 v7, a26
\tv_mfma_f32_16x16x32_bf16 a[28:31], v[8:11], a[88:91], a[28:31]
\tv_exp_f32_e32 v9, v40
\tds_read_b128 v[8:11], v50
\tv_add_f32_e32 v60, 1.0, v61
.Lfunc_end0:
"""


def test_mfma_war_flags_accumulator_read_and_source_overwrite(tmp_path, capsys):
    war = _load()
    p = tmp_path / "k.s"
    p.write_text(ASM)
    n = war.check(str(p), 4)
    out = capsys.readouterr().out
    # the accumulator read (a26 of a[24:27]) and the v9 write into SrcA v[8:11]; the ds_read
    # (lands long after issue) and the unrelated add are not hazards
    assert n == 2, out
    assert "v_accvgpr_read_b32 v7, a26" in out and "v_exp_f32_e32 v9" in out
    assert "v_add_f32" not in out and "ds_read" not in out.split("||")[-1]


def test_mfma_war_window(tmp_path):
    war = _load()
    p = tmp_path / "k.s"
    p.write_text(ASM)
    assert war.check(str(p), 1) == 1  # only the exp at distance 1 from the second MFMA


def _load_gen_report():
    spec = importlib.util.spec_from_file_location("gen_report", os.path.join(ROOT, "tools", "gen_report.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gen_report_writes_every_config_of_one_bench_line(tmp_path, monkeypatch):
    """tools/gen_report.py: the BASELINE.md / README.md tables come from ONE bench.py line (the
    headline and its "secondary" configs), replacing only the text between the markers."""
    import json
    import sys

    g = _load_gen_report()
    line = {"metric": "rows/sec", "value": 1929794.7, "n_gpus": 1, "steps": 20, "warmup": 5,
            "ms_per_step": 4.245, "dtype": "bf16", "data": "synthetic",
            "config": {"per_gpu_batch": 8192, "global_batch": 8192}, "persistent_fwd": True,
            "secondary": {"mlp": {"value": 1.0856e9, "ms_per_step": 0.2415, "per_gpu_batch": 262144,
                                  "steps": 20, "warmup": 5}}}
    src = tmp_path / "bench.log"
    src.write_text("noise\n" + json.dumps(line) + "\n")
    doc = tmp_path / "DOC.md"
    doc.write_text(f"head\n{g.BEGIN}\nold\n{g.END}\ntail\n")
    monkeypatch.setattr(sys, "argv", ["gen_report.py", str(src), "--write", str(doc)])
    assert g.main() == 0
    out = doc.read_text()
    assert out.startswith("head\n") and out.endswith("\ntail\n") and "old" not in out
    assert "| **LSTM seq64 h512 (headline)** | 8,192 | **1.930 M** | 4.245 | 20 (5) |" in out
    assert "| Static MLP 16-256-256-1 | 262,144 | 1.086 G | 0.241 | 20 (5) |" in out
    # a document without the markers is refused, not appended to
    bad = tmp_path / "BAD.md"
    bad.write_text("no markers\n")
    monkeypatch.setattr(sys, "argv", ["gen_report.py", str(src), "--write", str(bad)])
    assert g.main() == 1 and bad.read_text() == "no markers\n"
