"""Command line of the prof stage (reference apex/pyprof/prof/usage.py)."""
import argparse
import sys

from .output import COLUMNS, DEFAULT


def _cols(value):
    cols = value.split(",")
    bad = [c for c in cols if c not in COLUMNS]
    if bad:
        raise argparse.ArgumentTypeError("{} not valid; choose from {}".format(",".join(bad), ",".join(COLUMNS)))
    return cols


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="python -m apex.pyprof.prof",
                                 description="per-kernel FLOP / byte / MFMA report from apex.pyprof.parse output",
                                 formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("file", nargs="?", default=None, help="output of `python -m apex.pyprof.parse` (default stdin)")
    ap.add_argument("-c", type=_cols, default=DEFAULT,
                    help="comma separated columns:\n" + "\n".join("{:<8} {}".format(k, v[0])
                                                                 for k, v in COLUMNS.items()))
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--csv", action="store_true", help="CSV output")
    g.add_argument("-w", type=int, default=0, help="width of the columned output")
    ap.add_argument("--summary", choices=("op", "kName", "mod", "layer"), default=None,
                    help="print an aggregate table per op / kernel / module / layer instead")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args(argv)
    if isinstance(a.c, str):
        a.c = _cols(a.c)
    a.file = sys.stdin if a.file in (None, "-") else open(a.file)
    return a
