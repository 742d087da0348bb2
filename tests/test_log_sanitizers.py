"""The native log reader (csrc/pekf_log.cpp: host code that parses untrusted text) under AddressSanitizer
and UndefinedBehaviorSanitizer: tests/native/log_harness.cpp, built here with g++ against the reader's
source, scans and reads well-formed logs (pauses, a clock stepping back, lines of any length) and broken
ones (truncated, a missing value, no colon, binary bytes, empty, absent) without a sanitizer report,
with the results the library reports.  The same for the phone's wire text (csrc/pekf_wire.cpp,
tests/native/wire_harness.cpp): pekf_wire_parse on good, truncated, malformed and binary input, and
pekf_f32_wire_values over every class of float."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from poseestimationkf_amd import logformat, synth

from .conftest import ROOT


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = tmp_path_factory.mktemp("asan") / "log_harness"
    cmd = ["g++", "-g", "-O1", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "native", "log_harness.cpp"),
           os.path.join(ROOT, "poseestimationkf_amd", "csrc", "pekf_log.cpp"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return str(out)


def _logs(d):
    rng = np.random.default_rng(5)
    n = 120
    ts = np.cumsum(np.r_[1e12, rng.integers(4_000_000, 20_000_000, n)]).astype(np.float64)
    ts[40:] += 5e9          # a 5 s pause
    ts[70:] -= 3e7          # the clock steps back
    g, a, m = rng.normal(size=(3, n, 3))
    good = d / "good.txt"
    logformat.write_log(str(good), ts, g, a, m, [0, 0, 1.0], [0.5, 0, -0.8])
    lines = good.read_text().splitlines(keepends=True)
    files = {"good": good}
    files["trunc"] = d / "trunc.txt"
    files["trunc"].write_text("".join(lines[:len(lines) // 2]))
    bad = list(lines)
    i = next(k for k, l in enumerate(bad) if l.startswith("Acc_1"))
    bad[i] = "Acc_1 : 1.0,,2\n"
    files["missing_value"] = d / "missing_value.txt"
    files["missing_value"].write_text("".join(bad))
    long = list(lines)
    long[3] = "X_k : " + ", ".join(["1.0"] * 4000) + "\n"
    files["long_lines"] = d / "long_lines.txt"
    files["long_lines"].write_text("".join(long))
    files["no_colon"] = d / "no_colon.txt"
    files["no_colon"].write_text("gyro 1 2 3\nT\n")
    files["binary"] = d / "binary.bin"
    files["binary"].write_bytes(bytes(range(256)) * 40)
    files["empty"] = d / "empty.txt"
    files["empty"].write_text("")
    files["absent"] = d / "absent.txt"
    return files


def test_log_reader_under_sanitizers(harness, tmp_path):
    files = _logs(tmp_path)
    r = subprocess.run([harness] + [str(p) for p in files.values()], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    report = r.stdout + r.stderr
    assert r.returncode == 0 and "Sanitizer" not in report and "runtime error" not in report, report[-3000:]
    got = dict(zip(files, r.stdout.splitlines()))
    for name in ("good", "long_lines"):
        assert "scan=0 records=120 ext=0 escaped=2 plain=1 over=1 r64=0 over64=1" in got[name], got[name]
        assert " write=0 rescan=0 records=120" in got[name], got[name]
    assert " scan=0 " in got["trunc"] and " ext=0 " in got["trunc"] and " r64=0 " in got["trunc"]
    for name in ("missing_value", "no_colon", "binary", "empty", "absent"):
        assert " scan=1 " in got[name], got[name]


@pytest.fixture(scope="module")
def wire_harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = tmp_path_factory.mktemp("asan_wire") / "wire_harness"
    cmd = ["g++", "-g", "-O1", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "native", "wire_harness.cpp"),
           os.path.join(ROOT, "poseestimationkf_amd", "csrc", "pekf_wire.cpp"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return str(out)


def test_wire_parser_under_sanitizers(wire_harness, tmp_path):
    from poseestimationkf_amd import wire
    ev = synth.generate_events(np.arange(1), 60, seed=3)
    good = wire.events_text(ev["types"][:, 0], ev["values"][:, 0], ev["times"][:, 0])
    files = {"good": good, "trunc": good[: len(good) // 2 + 37], "no_newline": good.rstrip("\n"),
             "noise": "hello\n#\n#3\n" + "x" * 200 + "\n" + good,
             "missing_comma": "#3,0:1.5 2.5 3.5,t:12345" + " " * 60 + "\n",
             "missing_t": "#3,0:1.5,2.5,3.5," + " " * 60 + "\n",
             "bad_number": "#3,0:abc,2.5,3.5,t:12" + " " * 60 + "\n",
             "long_line": "#3,1:1." + "0" * 20000 + "1,2,3,t:5\n",
             "overflow": "#3,1:" + "1" * 400 + ",2,3,t:5\n", "empty": ""}
    paths = []
    for name, text in files.items():
        p = tmp_path / (name + ".txt")
        p.write_text(text)
        paths.append(str(p))
    p = tmp_path / "binary.bin"                          # no line starts with '#': nothing for the server
    p.write_bytes(bytes(range(256)) * 40)
    paths.append(str(p))
    p = tmp_path / "binary_hash.bin"                     # a '#' line of 245 garbage bytes: not a message
    p.write_bytes(b"\n#" + bytes(range(11, 256)) + b"\n")
    paths.append(str(p))
    r = subprocess.run([wire_harness] + paths, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    report = r.stdout + r.stderr
    assert r.returncode == 0 and "Sanitizer" not in report and "runtime error" not in report, report[-3000:]
    got = dict(zip(list(files) + ["binary", "binary_hash"], r.stdout.splitlines()))
    assert " scan=0 messages=60 full=0 under=1 " in got["good"], got["good"]
    assert " scan=0 messages=60 full=0 " in got["no_newline"] and " scan=0 messages=60 " in got["noise"]
    assert " scan=0 messages=0" in got["empty"] and " scan=0 messages=0" in got["binary"]
    # a message cut short (or malformed) is an error, where the server's std::stod / std::stoll would throw
    # (a value past the double range: std::stod's out_of_range)
    for name in ("trunc", "missing_comma", "missing_t", "bad_number", "binary_hash", "overflow"):
        assert " scan=1 " in got[name], (name, got[name])
    assert " scan=0 messages=1 full=0 " in got["long_line"], got["long_line"]
    last = r.stdout.splitlines()[-1]
    n = int(last.split("n=")[1].split()[0])
    assert last.startswith("f32_wire_values=0 ") and last.endswith("roundtrip=%d" % n), last
