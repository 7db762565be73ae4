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
