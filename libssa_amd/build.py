"""Builds the native libraries in-tree for gfx950: ``python -m libssa_amd.build``."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 8, quiet: bool = False) -> None:
    out = subprocess.DEVNULL if quiet else None
    subprocess.check_call(["make", "-C", HERE, f"-j{jobs}"], stdout=out)


if __name__ == "__main__":
    build(quiet="-q" in sys.argv)
