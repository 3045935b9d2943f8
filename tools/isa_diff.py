"""Compare the device code of kernels between two hipcc --cuda-device-only -S outputs.

    python tools/isa_diff.py old.s new.s [substring ...]

For every kernel (amdhsa function) whose mangled name contains one of the substrings (all kernels
by default) and exists in both files, the instruction streams are compared after normalising
per-function label numbers and dropping comments; prints one line per kernel (same / DIFFERENT /
only in one file).  Used to check that removing probe-only template branches leaves the launched
kernels bit-for-bit the same code."""
import re
import sys


def kernels(path):
    out, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r"^([_A-Za-z0-9.$]+):\s*(;.*)?$", line)
        if m and not line.startswith(".L") and cur is None and not m.group(1).startswith("."):
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                out[name] = cur
                cur = None
                continue
            t = line.split(";")[0].strip()
            if not t or t.startswith(".p2align") or t.startswith(".loc") or t.startswith(".cfi"):
                continue
            t = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", t)
            cur.append(t)
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    subs = sys.argv[3:]
    names = sorted(set(a) | set(b))
    bad = 0
    for n in names:
        if subs and not any(s in n for s in subs):
            continue
        if n not in a or n not in b:
            print(f"only in {'new' if n in b else 'old'}: {n}")
            continue
        same = a[n] == b[n]
        bad += not same
        print(f"{'same' if same else 'DIFFERENT'} ({len(a[n])} / {len(b[n])} lines): {n}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
