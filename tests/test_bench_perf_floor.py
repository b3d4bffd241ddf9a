"""bench.py's perf floor (tests/golden/perf_floor.json): every figure path
names a key the default line carries, and perf_summary reports a figure past
its limit as a PERF-REGRESSION line without failing the run. CPU only."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
FLOOR = json.load(open(os.path.join(HERE, "golden", "perf_floor.json")))


def _line():
    """A default-shaped line with every floor figure at its limit."""
    line = {"golden": {"c3": "match", "c2": "match"}}
    for name, spec in FLOOR.items():
        if name.startswith("_"):
            continue
        d = line
        for k in spec["path"][:-1]:
            d = d.setdefault(k, {})
        d[spec["path"][-1]] = spec.get("max", spec.get("min"))
    return line


def test_floor_specs_are_well_formed():
    for name, spec in FLOOR.items():
        if name.startswith("_"):
            continue
        assert isinstance(spec["path"], list) and spec["path"], name
        assert ("max" in spec) != ("min" in spec), name


def test_summary_at_the_limits_reports_nothing(capsys):
    import bench
    line = _line()
    bench.perf_summary(line)
    err = capsys.readouterr().err
    assert "SUMMARY" in err and "golden=2/2" in err
    assert "PERF-REGRESSION" not in err
    assert line["perf_check"]["regressions"] == []
    assert line["perf_check"]["checked"] == sum(1 for k in FLOOR if not k.startswith("_"))


def test_summary_flags_a_slower_figure(capsys):
    import bench
    line = _line()
    line["c5_multiarea_ksp2_ucmp"]["ms_per_step"] = 0.674  # the round-5 driver figure
    line["c5_multiarea_ksp2_ucmp"]["overlap"] = 0.99
    bench.perf_summary(line)
    err = capsys.readouterr().err
    assert "PERF-REGRESSION: c5_job_ms = 0.674" in err
    assert "PERF-REGRESSION: c5_overlap = 0.99" in err
    assert len(line["perf_check"]["regressions"]) == 2


def test_summary_skips_missing_figures(capsys):
    import bench
    line = {"golden": {}, "ms_per_step": 2.0}
    bench.perf_summary(line)
    err = capsys.readouterr().err
    assert "PERF-REGRESSION: c3_ms = 2" in err
    assert line["perf_check"]["checked"] == 1
