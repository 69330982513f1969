#!/usr/bin/env python3
"""Resolve tools/libsampler.so samples (gpurun_out/host_samples.txt) against
the libraries of this image: self and inclusive sample shares per function.
Usage: tools/sampler_report.py [samples.txt] [--top N]"""
import bisect
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    samples, maps = [], []
    for line in open(path):
        if line.startswith("S"):
            samples.append([int(x, 16) for x in line.split()[1:]])
        elif line.startswith("M "):
            f = line[2:].split()
            if len(f) >= 6:
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                maps.append((lo, hi, int(f[2], 16), f[5]))
    return samples, maps


LIBDIR = None  # directory holding the sampled run's copy of libpsf.so (host_samples_libpsf.so)


class Symbols:
    def __init__(self, path):
        self.addrs, self.names = [], []
        local = path
        if LIBDIR and os.path.basename(path) == "libpsf.so" and os.path.exists(os.path.join(LIBDIR, "host_samples_libpsf.so")):
            path = os.path.join(LIBDIR, "host_samples_libpsf.so")
            local = path
        if "/gpurun" in path or "graft" in path or not os.path.exists(path):
            base = os.path.basename(path)
            for cand in (os.path.join(ROOT, "parameter_server_amd", base), os.path.join(ROOT, "tools", base)):
                if os.path.exists(cand):
                    local = cand
        if not os.path.exists(local):
            return
        for opt in (["-C", "-n", "--defined-only"], ["-C", "-n", "-D", "--defined-only"]):
            out = subprocess.run(["nm", *opt, local], capture_output=True, text=True).stdout
            for ln in out.splitlines():
                p = ln.split(" ", 2)
                if len(p) == 3 and p[1] in "tTwW":
                    self.addrs.append(int(p[0], 16))
                    self.names.append(p[2])
            if self.addrs:
                break
        z = sorted(zip(self.addrs, self.names))
        self.addrs = [a for a, _ in z]
        self.names = [n for _, n in z]

    def name(self, v):
        i = bisect.bisect_right(self.addrs, v) - 1
        return self.names[i] if i >= 0 else "?"


def main():
    argv = sys.argv[1:]
    if "--top" in argv:
        i = argv.index("--top")
        argv = argv[:i] + argv[i + 2:]
    args = [a for a in argv if not a.startswith("--")]
    top = 40
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    path = args[0] if args else os.path.join(ROOT, "gpurun_out", "host_samples.txt")
    global LIBDIR
    LIBDIR = os.path.dirname(os.path.abspath(path))
    samples, maps = load(path)
    base = {}
    for lo, hi, off, p in maps:
        if off == 0 and p not in base:
            base[p] = lo
    syms = {}

    def resolve(a):
        for lo, hi, off, p in maps:
            if lo <= a < hi:
                if p not in syms:
                    syms[p] = Symbols(p)
                s = syms[p]
                v = a - base.get(p, lo)
                short = os.path.basename(p)
                return f"{s.name(v)} [{short}]"
        return "?"

    cache = {}
    selfc, incl = collections.Counter(), collections.Counter()
    for fr in samples:
        names = []
        for d, a in enumerate(fr):
            if d == 1:
                continue  # the signal trampoline / handler frame
            if a not in cache:
                cache[a] = resolve(a - (1 if d > 1 else 0))
            names.append(cache[a])
        if not names:
            continue
        names = names[1:] if "on_prof" in names[0] else names
        if not names:
            continue
        selfc[names[0]] += 1
        for nm in set(names):
            incl[nm] += 1
    n = len(samples)
    print(f"{n} samples")
    print("--- self")
    for nm, c in selfc.most_common(top):
        print(f"{100 * c / n:6.2f}%  {nm[:150]}")
    print("--- inclusive (any of the first frames)")
    for nm, c in incl.most_common(top):
        print(f"{100 * c / n:6.2f}%  {nm[:150]}")




def by_first_own_frame(path, lib="libpsf", top=30):
    """samples charged to the innermost frame in `lib` (its own time plus the
    library / runtime calls it makes); samples with no such frame in the
    recorded depth are counted as '(deeper)'"""
    global LIBDIR
    LIBDIR = os.path.dirname(os.path.abspath(path))
    samples, maps = load(path)
    base = {}
    for lo, hi, off, p in maps:
        if off == 0 and p not in base:
            base[p] = lo
    syms = {}
    cache = {}
    c = collections.Counter()
    for fr in samples:
        name = "(deeper)"
        for d, a in enumerate(fr[2:]):
            if a not in cache:
                cache[a] = None
                for lo, hi, off, p in maps:
                    if lo <= a - 1 < hi and lib in p:
                        if p not in syms:
                            syms[p] = Symbols(p)
                        cache[a] = syms[p].name(a - 1 - base.get(p, lo))
                        break
            if cache[a]:
                name = cache[a]
                break
        c[name] += 1
    n = len(samples)
    for nm, k in c.most_common(top):
        print(f"{100 * k / n:6.2f}%  {nm[:160]}")


if __name__ == "__main__":
    if "--own" in sys.argv:
        a = [x for x in sys.argv[1:] if not x.startswith("--")]
        by_first_own_frame(a[0] if a else os.path.join(ROOT, "gpurun_out", "host_samples.txt"))
    else:
        main()
