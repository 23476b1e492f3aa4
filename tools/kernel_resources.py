"""Per-kernel register / spill / LDS use of the gfx950 code objects in libmrl_hip.so
(from the code-object metadata notes).  usage: python tools/kernel_resources.py [substr ...]"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_hazard_check import LLVM, code_objects  # noqa: E402

FIELDS = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size",
          "private_segment_fixed_size")


def kernels(lib):
    out = []
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", f.name], capture_output=True,
                                   text=True).stdout
        for ent in re.split(r"\n\s+- \.", notes):
            m = re.search(r"\.name:\s+(\S+)", ent)
            if not m or ".vgpr_count" not in ent:
                continue
            vals = {}
            for k in FIELDS:
                mm = re.search(r"\." + k + r":\s+(\d+)", ent)
                vals[k] = int(mm.group(1)) if mm else None
            out.append((m.group(1), vals))
    return out


def main():
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "modular_rl_amd", "libmrl_hip.so")
    pats = sys.argv[1:]
    for name, v in kernels(lib):
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name[:90]:90s} v{v['vgpr_count']} a{v['agpr_count']} spill{v['vgpr_spill_count']} "
              f"lds{v['group_segment_fixed_size']} scratch{v['private_segment_fixed_size']}")


if __name__ == "__main__":
    main()
