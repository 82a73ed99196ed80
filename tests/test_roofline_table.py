"""tools/roofline_table.py prices each kernel's algorithmic bytes with the
counts of a bench line, not with constants."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("roofline_table", os.path.join(ROOT, "tools", "roofline_table.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _line(L):
    return {"metric": "x", "config": {"gaussians": 1000, "visible": 900, "tile_touches": 5000,
                                      "records_consumed": 3000, "live_entry_cells": L, "width": 64, "height": 48}}


def test_counts_come_from_the_bench_line(tmp_path):
    rt = _tool()
    src = open(os.path.join(ROOT, "tools", "roofline_table.py")).read()
    assert "11_540_000" not in src and "4_411_397" not in src  # (the round-5 constants)
    pmc = tmp_path / "pmc.txt"
    pmc.write_text("# library_source_sha256 abc\nk_gather_slots\n  FETCH_SIZE 100\n  WRITE_SIZE 50\n"
                   "k_blend_bwd\n  FETCH_SIZE 10\n  WRITE_SIZE 5\n")
    stats = tmp_path / "stats.txt"
    stats.write_text("k_gather_slots<4, 2, 4>  20  10.0\nk_blend_bwd<true, false>  20  100.0\n")
    for L in (1234, 98765):
        log = tmp_path / f"bench{L}.log"
        log.write_text("progress line\n" + json.dumps(_line(L)) + "\n")
        k = rt.counts_from_bench(rt.bench_line(str(log)))
        assert k == {"N": 1000, "M": 900, "T": 5000, "R": 3000, "L": L, "HW": 64 * 48, "TILES": 4 * 3}
        out = rt.table(rt.pmc(str(pmc)), rt.timed(str(stats)), k)
        row = [r for r in out.splitlines() if r.startswith("k_gather_slots")][0].split()
        assert float(row[3]) == round((40 * L + 4 * 5000 + 40 * 1000) / 1e6, 1)
        bwd = [r for r in out.splitlines() if r.startswith("k_blend_bwd")][0].split()
        assert float(bwd[3]) == round((44 * 3000 + 36 * 64 * 48 + 40 * 900) / 1e6, 1)
        assert f"L={L:,}" in out.splitlines()[0]
