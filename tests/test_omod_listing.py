"""The exact halvings that ride on VOP3 output modifiers (omod div:2 / mul:2 / mul:4, pekf_math.hpp
fma_half & co.) only take effect inside the MODE window OmodMode opens (IEEE off, FP64 denormals
flushed); outside it the hardware silently ignores the modifier and the result is off by 2x.  The
inline asm of those helpers is ordered only by its data dependences, so this checks the emitted gfx950
listing of every kernel that uses them (the multi-record k_run variants and k_live): each omod
instruction lies between the window's MODE write and the write that restores the saved MODE, in the
same function.  CPU only (hipcc cross-compiles); ADVICE r2."""
import os
import re
import shutil
import subprocess

import pytest

from .conftest import ROOT

CSRC = os.path.join(ROOT, "poseestimationkf_amd", "csrc")
COMMON = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
          "-fno-slp-vectorize", "-ffp-contract=on", "--cuda-device-only", "-S"]
OMOD = re.compile(r"\s(div:2|mul:2|mul:4)\b")
GETREG = re.compile(r"s_getreg_b32\s+(s\d+),\s*hwreg\(HW_REG_MODE,\s*6,\s*4\)")
SETREG = re.compile(r"s_setreg_b32\s+hwreg\(HW_REG_MODE,\s*6,\s*4\),\s*(s\d+)")


def _listing(src, extra, tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([hipcc] + COMMON + extra + [os.path.join(CSRC, src), "-o", str(out)], check=True,
                   capture_output=True, timeout=600)
    return out.read_text().splitlines()


def _functions(lines):
    """{name: [lines]} of the kernels in a listing (label line to .Lfunc_end)."""
    fns, cur = {}, None
    for raw in lines:
        line = raw.split(";")[0].rstrip()
        m = re.match(r"^([_A-Za-z][\w.$]*):\s*$", line)
        if m and not line.startswith(".L") and line.startswith("_Z"):
            cur = fns.setdefault(m.group(1), [])
            continue
        if cur is not None:
            if line.strip().startswith(".Lfunc_end"):
                cur = None
                continue
            cur.append(line)
    return fns


def _check_function(body):
    """CFG dataflow over one kernel: the MODE window's state (open / closed) at every instruction, over
    all paths (basic blocks split at .LBB labels, successors from s_branch / s_cbranch_* and fall
    through).  Returns the number of omod instructions; asserts each is reached only with the window
    open."""
    blocks, order, cur = {}, [], "entry"
    blocks[cur], order = [], [cur]
    for line in body:
        m = re.match(r"^(\.LBB[\w]+):", line)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        if line.strip() and not line.strip().startswith("."):
            blocks[cur].append(line.strip())
    saved = {m.group(1) for l in body for m in [GETREG.search(l)] if m}
    succ = {}
    for i, b in enumerate(order):
        ins = blocks[b]
        nxt = order[i + 1] if i + 1 < len(order) else None
        last = ins[-1] if ins else ""
        out = []
        for l in ins:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)", l)
            if m:
                out.append(m.group(1))
        m = re.match(r"s_branch\s+(\.LBB\w+)", last)
        if m:
            out.append(m.group(1))
        elif not last.startswith("s_endpgm") and nxt is not None:
            out.append(nxt)
        succ[b] = out

    def transfer(b, state, check=False):
        n = 0
        for l in blocks[b]:
            m = SETREG.search(l)
            if m:
                state = {False} if m.group(1) in saved else {True}
            elif OMOD.search(" " + l) and l.startswith("v_"):
                n += 1
                if check:
                    assert state == {True}, "omod instruction reachable outside the MODE window: %s" % l
        return state, n

    entry_state = {b: set() for b in order}
    entry_state["entry"] = {False}
    work = ["entry"]
    while work:
        b = work.pop()
        out, _ = transfer(b, set(entry_state[b]))
        for s_ in succ[b]:
            if not out <= entry_state[s_]:
                entry_state[s_] |= out
                work.append(s_)
    return sum(transfer(b, set(entry_state[b]), check=True)[1] for b in order if entry_state[b])


def _check(lines):
    """(kernels with omod instructions, omod instructions) over a listing, every one checked."""
    n_fn = n_omod = 0
    for name, body in _functions(lines).items():
        n = _check_function(body)
        n_fn += n > 0
        n_omod += n
    return n_fn, n_omod


def test_omod_only_inside_the_mode_window_multi_record(tmp_path):
    lines = _listing("pekf_run_multi.hip", ["-mllvm", "--amdgpu-sched-strategy=max-ilp"], tmp_path)
    n_fn, n_omod = _check(lines)
    assert n_fn >= 8 and n_omod > 1000      # every FP64 multi-record variant carries them


def test_omod_only_inside_the_mode_window_live(tmp_path):
    lines = _listing("pekf_live.hip", [], tmp_path)
    n_fn, n_omod = _check(lines)
    # k_live<TE, R64>: time events or not x FP64 / f32 records, and k_live<.., EV64> (FP64 events)
    assert n_fn == 5 and n_omod > 100


def test_checker_catches_an_omod_outside_the_window():
    """The dataflow sees through block layout: a restore placed textually before the window's opening
    (a loop) is fine, an omod reachable on a path with the window closed is not."""
    ok = ["s_getreg_b32 s26, hwreg(HW_REG_MODE, 6, 4)", ".LBB0_1:", "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s4",
          "v_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7] div:2", "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s26",
          "s_cbranch_vccnz .LBB0_1", "s_endpgm"]
    assert _check_function(ok) == 1
    loop_back = ["s_getreg_b32 s26, hwreg(HW_REG_MODE, 6, 4)", "s_branch .LBB0_2", ".LBB0_1:",
                 "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s26", "s_cbranch_vccz .LBB0_3", ".LBB0_2:",
                 "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s4", "v_mul_f64 v[0:1], v[2:3], v[4:5] div:2",
                 "s_branch .LBB0_1", ".LBB0_3:", "s_endpgm"]
    assert _check_function(loop_back) == 1
    bad = ["s_getreg_b32 s26, hwreg(HW_REG_MODE, 6, 4)", "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s4",
           "s_cbranch_execz .LBB0_1", "s_setreg_b32 hwreg(HW_REG_MODE, 6, 4), s26", ".LBB0_1:",
           "v_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7] div:2", "s_endpgm"]
    with pytest.raises(AssertionError, match="outside the MODE window"):
        _check_function(bad)
