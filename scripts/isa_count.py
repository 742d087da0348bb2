#!/usr/bin/env python3
"""Count instructions of one kernel in a hipcc -S listing, split into the hot loop and the rest.

usage: scripts/isa_count.py <file.s> <kernel-substring> [steps-per-iteration]
The hot loop is taken as the largest block between a label and a backward branch to it;
k_run's time loop is unrolled by two, so its counts are divided by 2 (the default).
"""
import collections
import re
import sys


def kernel_lines(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    return lines[start:end + 1]


LABEL = re.compile(r"^([.\w$]+):")


def is_insn(l):
    s = l.strip()
    return bool(s) and not s.startswith((";", ".", "//")) and not LABEL.match(s)


def main():
    path, name = sys.argv[1], sys.argv[2]
    spi = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    body = kernel_lines(path, name)
    labels = {LABEL.match(l.strip()).group(1): i for i, l in enumerate(body) if LABEL.match(l.strip())}
    best = (0, 0)
    for i, l in enumerate(body):
        m = re.match(r"\s*s_cbranch_\w+\s+(\S+)|\s*s_branch\s+(\S+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i and i - labels[tgt] > best[1] - best[0]:
                best = (labels[tgt], i)
    loop = [l.strip().split()[0] for l in body[best[0]:best[1] + 1] if is_insn(l)]
    allc = [l.strip().split()[0] for l in body if is_insn(l)]
    c = collections.Counter(loop)
    f64 = {k: v for k, v in c.items() if "_f64" in k}
    flops = sum(v * (2 if "fma" in k else 1) for k, v in f64.items()
                if any(t in k for t in ("fma", "mul_f64", "add_f64", "rcp", "rsq", "sqrt")))
    print("kernel instructions: %d, hot loop: %d (%d steps per iteration)" % (len(allc), len(loop), spi))
    print("loop FP64 VALU: %d  (%s)" % (sum(f64.values()), ", ".join("%s %d" % kv for kv in sorted(f64.items(), key=lambda x: -x[1]))))
    print("per filter-step: FP64 VALU %.1f, FP64 FLOP (fma=2; add/mul/rcp/rsq=1) %.1f, all VALU %.1f"
          % (sum(f64.values()) / spi, flops / spi, sum(v for k, v in c.items() if k.startswith("v_")) / spi))
    groups = collections.Counter()
    for k, v in c.items():
        g = ("v_f64" if "_f64" in k else "v_mfma" if "mfma" in k else "v_other" if k.startswith("v_")
             else "s_" if k.startswith("s_") else "global/buffer" if k.startswith(("global_", "buffer_")) else k)
        groups[g] += v
    print("loop groups:", dict(groups))
    print("top:", ", ".join("%s %d" % kv for kv in c.most_common(25)))


if __name__ == "__main__":
    main()
