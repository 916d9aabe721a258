"""CPU checks of bench.py's accounting (no GPU): which cost kernel a geometry /
palette size runs, its nominal and executed flops per pixel-evaluation (the
roofline line), the split choice for N > 1, and the committed HBM-traffic
lookup keyed on the configuration."""

import bench


def test_default_geometry_is_the_21_tap_fast_path():
    kernel, hb, chunked, nominal, executed = bench.cost_accounting(10, 256, 32, {})
    assert (kernel, hb, chunked) == ("cost16w_kernel", 10, False)
    assert nominal == 628  # 7 x 2 x 21 x 2 + 40
    assert executed == 2 * 2 * (4 * 21 + 7 + 9 + 11) + 40  # trimmed k1 windows: 484


def test_viewing_geometries_and_palette_sizes():
    assert bench.cost_accounting(19, 256, 32, {})[:2] == ("cost16w_kernel", 19)
    assert bench.cost_accounting(19, 256, 32, {})[3] == 7 * 2 * 39 * 2 + 40  # 1132
    assert bench.cost_accounting(20, 256, 32, {})[1] == 24  # bucket 24 holds H = 20
    k, hb, _, nominal, executed = bench.cost_accounting(51, 256, 32, {})  # 300 dpi / 50 cm
    assert (k, hb) == ("gen_hmfma_kernel+gen_vmfma_kernel", 0) and executed == 2 * 2 * 7 * 103 + 40
    assert bench.cost_accounting(10, 256, 32, {"cost_variant": 2})[0] == "gen_hpass_kernel+gen_vpass_kernel"
    assert bench.cost_accounting(10, 256, 32, {"cost_rows": 8})[0] == "cost_mfma_kernel"
    assert bench.cost_accounting(10, 1024, 32, {})[:3] == ("cost16w_kernel", 10, True)  # chunked
    assert bench.cost_accounting(19, 1024, 32, {})[1] == 0  # chunked runs HB = 10 only
    assert bench.cost_accounting(10, 5000, 32, {})[:3] == ("cost16w_kernel", 10, True)  # 32 chunks
    assert bench.cost_accounting(10, 10000, 32, {})[:3] == ("gen_hmfma_kernel+gen_vmfma_kernel", 0, True)  # 64
    assert bench.cost_accounting(10, 20000, 32, {})[:3] == ("gen_hmfma_kernel+gen_vmfma_kernel", 0, False)
    assert bench.cost_accounting(70, 256, 32, {})[0] == "gen_hrow4_kernel+gen_vtile_kernel"  # half > 64
    assert bench.cost_accounting(51, 256, 32, {"gen_hmfma": 0})[0] == "gen_hrow4_kernel+gen_vmfma_kernel"
    assert bench.cost_accounting(51, 256, 32, {"gen_vmfma": 0})[0] == "gen_hrow4_kernel+gen_vtile2_kernel"


def test_split_choice():
    assert not bench.use_palette_split("auto", 4, 1)
    assert not bench.use_palette_split("auto", 4, 8)  # C3: rows
    assert bench.use_palette_split("auto", 64, 8)  # C5 on 8 GPUs
    assert not bench.use_palette_split("auto", 64, 16) and not bench.use_palette_split("auto", 60, 8)
    assert bench.use_palette_split("palettes", 8, 2) and not bench.use_palette_split("rows", 64, 8)


def test_measured_traffic_lookup():
    t = bench.measured_traffic(4096, 256, 4, 32, 1, "cost16w_kernel")
    assert t is not None and 2.5e8 < t < 3.0e8  # the committed PMC passes (~271 MB per launch)
    assert bench.measured_traffic(4096, 256, 4, 32, 2, "cost16w_kernel") is None  # multi-GPU: none
    assert bench.measured_traffic(4096, 256, 4, 32, 1, "cost16w_kernel", dpi=96, distance=60.0) is None


def test_measured_traffic_takes_the_newest_matching_file(tmp_path, monkeypatch):
    """Any rNN*hbm_traffic.json counts; the newest round wins, then the latest
    `generated` stamp; an empty config never matches."""
    import json
    import os

    prof = tmp_path / "profiles"
    prof.mkdir()
    cfg = {"size": 4096, "K": 256, "P": 4, "grid": 32}

    def put(name, traffic, config, generated=None):
        d = {"config": config, "kernels": {"hq::cost16w_kernel<10, 0, true, 4, 1>": {"traffic_bytes": traffic}}}
        if generated:
            d["generated"] = generated
        (prof / name).write_text(json.dumps(d))

    put("r04_hbm_traffic.json", 100, cfg)
    put("r04_wave_acc_hbm_traffic.json", 200, {})  # no config: never matches
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.measured_traffic(4096, 256, 4, 32, 1, "cost16w_kernel") == 100
    put("r05_a_hbm_traffic.json", 300, cfg, "2026-10-18T10:00:00Z")
    put("r05_b_hbm_traffic.json", 400, cfg, "2026-10-18T09:00:00Z")
    assert bench.measured_traffic(4096, 256, 4, 32, 1, "cost16w_kernel", with_source=True) == \
        (300, "r05_a_hbm_traffic.json")
    assert bench.measured_traffic(4096, 256, 8, 32, 1, "cost16w_kernel") is None
    assert os.path.basename(str(tmp_path))  # (ROOT restored by monkeypatch)


def test_profile_stages_and_single_rank_line():
    assert "comm" not in bench.profiled_stages(1) and bench.profiled_stages(2)[-1] == "comm"
    avg, mx = bench.kernel_profile({"cost": (0.35, 100), "assign": (0.15, 100)}, 1)
    assert avg == {"cost": 0.35, "assign": 0.15} and mx is None
