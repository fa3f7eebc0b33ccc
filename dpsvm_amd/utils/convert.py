"""Dataset converters (reference scripts/, Python 2 -> 3).

  mnist:  convert_mnist_to_odd_even.py:5-31  label parity -> +1 (even) / -1 (odd),
          pixels / 255.
  adult:  convert_adult.py:5-35  a9a LIBSVM sparse -> dense 0/1 CSV.  The
          reference writes feature k into column k+1 of a 124-wide row, so
          column 1 is always 0 and k = 123 overflows.  Default here:
          feature k -> feature column k (1-based), d = 123.  ``legacy_shift``
          reproduces the reference layout (d = 124 with the empty column; k=123
          is dropped instead of crashing).

CLI:  python -m dpsvm_amd.utils.convert mnist mnist_train.csv [out.csv]
      python -m dpsvm_amd.utils.convert adult a9a.txt [out.csv] [--legacy-shift]
"""
from __future__ import annotations

import argparse
import sys


def _default_out(path: str) -> str:
    return path[: len(path) - 4] + "_conv.csv"  # reference naming (both scripts, line 8)


def convert_mnist(src: str, dst: str | None = None) -> str:
    dst = dst or _default_out(src)
    with open(src) as fi, open(dst, "w") as fo:
        for line in fi:
            line = line.strip()
            if not line:
                continue
            tok = line.split(",")
            lab = "1" if int(float(tok[0])) % 2 == 0 else "-1"
            fo.write(",".join([lab] + [repr(float(t) / 255.0) for t in tok[1:]]) + "\n")
    return dst


def convert_adult(src: str, dst: str | None = None, legacy_shift: bool = False, d: int = 123) -> str:
    dst = dst or _default_out(src)
    with open(src) as fi, open(dst, "w") as fo:
        for line in fi:
            line = line.strip()
            if not line:
                continue
            tok = line.split()
            lab = "-1" if tok[0].startswith("-") else "1"
            if legacy_shift:
                # reference: 124 tokens, token 0 = label, feature k -> token k+1
                row = ["0"] * 124
                row[0] = lab
                for t in tok[1:]:
                    k = int(t.split(":")[0])
                    if k + 1 < 124:
                        row[k + 1] = "1"
            else:
                row = [lab] + ["0"] * d
                for t in tok[1:]:
                    k = int(t.split(":")[0])
                    if 1 <= k <= d:
                        row[k] = "1"
            fo.write(",".join(row) + "\n")
    return dst


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="dpsvm dataset converters")
    ap.add_argument("kind", choices=["mnist", "adult"])
    ap.add_argument("src")
    ap.add_argument("dst", nargs="?")
    ap.add_argument("--legacy-shift", action="store_true")
    a = ap.parse_args(argv)
    print("Processing ...")
    out = convert_mnist(a.src, a.dst) if a.kind == "mnist" else convert_adult(a.src, a.dst, a.legacy_shift)
    print(f"Done -> {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
