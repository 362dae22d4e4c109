#!/usr/bin/env python3
"""Register / spill metadata of the kernels in a hipcc device assembly file (-S
--cuda-device-only, or -save-temps' *-gfx950.s): one line per kernel whose name matches the
filter (substring of the mangled name).

    python tools/kmeta.py build.s [k_env_step_pair]"""
import sys

import yaml


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    txt = open(path).read()
    a = txt.index("amdhsa.kernels:")
    b = txt.index(".end_amdgpu_metadata")
    doc = yaml.safe_load("---\n" + txt[a:b].replace("\t", "  "))
    for k in doc["amdhsa.kernels"]:
        if filt and filt not in k[".name"]:
            continue
        print(f"{k['.name'][:70]:70s} vgpr {k.get('.vgpr_count')} agpr {k.get('.agpr_count')} "
              f"sgpr {k.get('.sgpr_count')} vspill {k.get('.vgpr_spill_count')} "
              f"sspill {k.get('.sgpr_spill_count')} scratch {k.get('.private_segment_fixed_size')} "
              f"lds {k.get('.group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
