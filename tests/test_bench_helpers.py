"""CPU checks of bench.py's own arithmetic: the timeline reader behind the
answer roofline's `union` figure and the query phase's busy share."""
import importlib.util
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("pm_bench", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_read_timeline_union_and_busy(tmp_path):
    f = tmp_path / "tl.csv"
    # two overlapping answers (union 150 us of 200 summed), a gap, maintenance after 300 us
    f.write_text("answer,0,100,0x1\n"
                 "answer,50,150,0x2\n"
                 "match_resolve,150,170,0x1\n"
                 "team_round,170,200,0x1\n"
                 "prep_offsets,300,400,0x1\n"
                 "prep_fold,400,600,0x1\n")
    t = _bench().read_timeline(str(f))
    assert t["answer"] == {"launches": 2, "sum_ms": 0.2, "union_ms": 0.15}
    assert t["prep_fold"]["union_ms"] == 0.2
    qp = t["query_phase"]
    assert qp["ms"] == 0.3 and abs(qp["busy_frac"] - 200 / 300) < 1e-3


def test_read_timeline_no_maintenance(tmp_path):
    f = tmp_path / "tl.csv"
    f.write_text("answer,10,20,0x1\nanswer,30,40,0x1\n")
    t = _bench().read_timeline(str(f))
    assert t["answer"]["union_ms"] == 0.02 and "query_phase" not in t


def _run_watchdog(body: str):
    import json
    import subprocess
    import sys
    import time
    code = ("import importlib.util, sys, time\n"
            f"spec = importlib.util.spec_from_file_location('pm_bench', {str(ROOT / 'bench.py')!r})\n"
            "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n" + body)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, [json.loads(ln) for ln in lines], time.monotonic() - t0


def test_watchdog_writes_the_partial_line_and_exits():
    """A stuck multi-rank block: the watchdog writes the one line (the blocks
    marked unfinished, watchdog.fired) and ends the process with status 3,
    instead of a hang."""
    rc, lines, dt = _run_watchdog(
        "out = {'metric': 'm', 'value': 1.0}\n"
        "wd = b.Watchdog(out, 0, 1, 0.3)\n"
        "time.sleep(30)\n"
        "print('not reached')\n")
    assert rc == 3 and len(lines) == 1, (rc, lines)   # non-zero: the caller sees the hang
    assert lines[0]["value"] == 1.0
    assert "unfinished" in lines[0]["config3_bigann_100m"]["error"]
    assert lines[0]["watchdog"] == {"fired": True, "budget_s": 0.3}   # the hang is reported in the line
    assert dt < 25


def test_watchdog_snapshot_keeps_finished_blocks():
    """Blocks finished before the budget expired (Watchdog.put, under the
    watchdog's lock) are in the line; the one still running is marked."""
    rc, lines, _ = _run_watchdog(
        "out = {'metric': 'm', 'value': 3.0}\n"
        "wd = b.Watchdog(out, 0, 1, 0.5)\n"
        "wd.put('config3_bigann_100m', {'value': 7.0})\n"
        "time.sleep(30)\n")
    assert rc == 3 and len(lines) == 1, (rc, lines)
    assert lines[0]["config3_bigann_100m"] == {"value": 7.0}
    assert "unfinished" in lines[0]["config4_bigann_1b"]["error"]
    assert lines[0]["watchdog"]["fired"] is True


def test_watchdog_fire_before_the_budget():
    rc, lines, _ = _run_watchdog(
        "out = {'metric': 'm', 'value': 2.0}\n"
        "wd = b.Watchdog(out, 0, 1, 5.0)\n"
        "assert wd.fire() is True\n"
        "assert wd.fire() is False\n"
        "import json; print(json.dumps({'finished': True}))\n")
    assert rc == 0 and lines == [{"finished": True}]
