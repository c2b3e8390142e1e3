"""Compare the gfx950 machine code of kernels between two device assembly files (hipcc --cuda-device-only -S):
a source refactor that must not change the product kernels is checked by
  python tools/asm_diff.py before.s after.s [kernel-substring ...]
Each kernel's body (label to .Lfunc_end) is normalised (local labels renumbered in order of appearance,
comments and blank lines dropped) and compared instruction for instruction; kernels present in only one
file are listed. Exit status 1 when a compared kernel differs."""
import re
import subprocess
import sys


def kernels(path):
    out, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and cur is None:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                out[name] = cur
                cur = None
                continue
            s = line.split(";")[0].rstrip()
            if s.strip():
                cur.append(s.strip())
    return out


def normalise(body):
    labels = {}
    res = []
    for s in body:
        for lab in re.findall(r"\.L[A-Za-z_0-9]+", s):
            labels.setdefault(lab, f".L{len(labels)}")
        res.append(re.sub(r"\.L[A-Za-z_0-9]+", lambda m: labels[m.group(0)], s))
    return res


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return dict(zip(names, p.stdout.splitlines())) if p.returncode == 0 else {n: n for n in names}


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    pats = sys.argv[3:]
    dm = demangle(sorted(set(a) | set(b)))
    sel = lambda n: not pats or any(p in dm[n] for p in pats)
    bad = 0
    for n in sorted(set(a) | set(b), key=lambda n: dm[n]):
        if not sel(n):
            continue
        if n not in a or n not in b:
            print(f"{'only in ' + ('first' if n in a else 'second'):16s} {dm[n]}")
            continue
        na, nb = normalise(a[n]), normalise(b[n])
        same = na == nb
        bad += not same
        print(f"{'same' if same else 'DIFFERENT':16s} {dm[n]} ({len(na)} / {len(nb)} lines)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
