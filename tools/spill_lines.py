#!/usr/bin/env python3
"""Scratch (spill) stores / loads and SGPR-spill lane moves of one kernel of a hipcc device
assembly file built with -gline-tables-only, per source line.

    python tools/spill_lines.py build.s k_env_step_pairIN2mi6TopoCTINS0_13RobotHumanoid [top]"""
import collections
import re
import sys


FOCUS = "mi_pair.hpp"


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    files = {}
    cnt = collections.Counter()
    inside = False
    loc = "?"
    spill_vgprs = set()   # VGPRs that hold SGPR spills (destinations of v_writelane)
    for ln in open(path):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"(?:\s+\"([^\"]*)\")?", ln)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if not inside:
            if ln.startswith("_Z") and name in ln.split(":")[0]:
                inside = True
            continue
        if ln.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            # the innermost frame of the inline chain that lies in mi_pair.hpp (else the leaf)
            frames = re.findall(r"([\w.]+\.(?:hpp|hip|h)):(\d+):\d+", ln.split(";", 1)[-1])
            fr = [f for f in frames if f[0] == FOCUS]
            loc = f"{fr[0][0]}:{fr[0][1]}" if fr else f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        s = ln.strip()
        if s.startswith("scratch_store") or s.startswith("buffer_store_dword") and "off, s[0:3]" in s:
            cnt[("vstore", loc)] += 1
        elif s.startswith("scratch_load"):
            cnt[("vload", loc)] += 1
        elif s.startswith("v_writelane_b32"):
            cnt[("swritelane", loc)] += 1
            spill_vgprs.add(s.split()[1].rstrip(","))
        elif s.startswith("v_readlane_b32"):
            src = s.split()[2].rstrip(",")
            cnt[("sreload" if src in spill_vgprs else "readlane", loc)] += 1
    for (k, l), v in cnt.most_common(top):
        print(f"{k:11s} {l:24s} {v}")


if __name__ == "__main__":
    main()
