"""The asyncio debug-mode warnings (``Executing <…> took N seconds``) in the children's stderr
files (``gpu_pass.sh burstdebug``): process, time, callback, seconds — slowest last."""

import glob
import os
import re
import sys

PAT = re.compile(r'"ts":"([^"]+)".*?Executing (.*) took ([0-9.]+) seconds')
AT = re.compile(r"(?:coro=<|<Handle |<TimerHandle )([^>]*?) (?:running at|created at|at) ([^ >]+)")


def main(d: str) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "*.log")):
        for line in open(f, errors="replace"):
            mo = PAT.search(line)
            if mo:
                at = AT.search(mo.group(2))
                what = f"{at.group(1)} @ {at.group(2)}" if at else mo.group(2)[:160]
                rows.append((float(mo.group(3)), os.path.basename(f).split(".")[0], mo.group(1), what))
    for sec, proc, ts, what in sorted(rows)[-40:]:
        print(f"{proc:45s} {ts} {sec:7.3f}s {what}")


if __name__ == "__main__":
    main(sys.argv[1])
