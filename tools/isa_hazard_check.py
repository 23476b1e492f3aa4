"""Check the built gfx950 code objects of libmrl_hip.so for the packed-f32 -> LDS hazard.

DESIGN §3 (round 5): a v_pk_{fma,mul,add}_f32 result read as DATA by an LDS instruction
(ds_bpermute_b32 in head_finish's cross-half shuffle) one instruction later delivered
stale values for the last quarter of the wave (lanes 48-63) -- run to run, a few 16-row
groups per 4 M rows (tools/det_locate.py, gpurun_out/r05_det*.log).  hipcc pads a
packed-f32 write before a VALU consumer (s_nop 0) but not before an LDS consumer.  This
tool disassembles every gfx950 code object bundled in the library and reports each LDS
instruction that reads as data a VGPR written by a packed-f32 VALU op:
  * a cross-lane LDS read (ds_bpermute / ds_permute / ds_swizzle, the failing pattern)
    anywhere earlier in the same basic block -- no wait-state count is trusted there;
  * any other LDS data read (ds_write / ds_add ...) fewer than MIN_STATES = 8 wait states
    earlier: four times the two wait states (s_nop 1) proven insufficient by a build that
    still corrupted 1,024 rows (profiles/r05_det_slp_bpermute_nop.txt; one wait state:
    24.8-33.1 k rows).  The library's nearest such site is 12 states away
    (mlp_vjp_kernel's dtanh products into its LDS transposes; `--strict` lists them).
No ISA document available here states the hazard's window.
--min-states N replaces the 8; --strict applies the whole-block rule to every LDS read.

usage: python tools/isa_hazard_check.py [lib.so] [--min-states N | --strict] [--all]
exit status 1 if a hazard is found (tests/test_abi.py runs it on the built library)."""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MIN_STATES = 8  # wait states required before a non-permute LDS data read (None: whole block)
CROSS_LANE = ("ds_bpermute", "ds_permute", "ds_swizzle")  # whole-block rule always


def code_objects(lib):
    """gfx950 code objects of every offload bundle in the library's .hip_fatbin."""
    with tempfile.TemporaryDirectory() as td:
        sec = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, sec], check=True)
        data = open(sec, "rb").read()
    out, pos = [], data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple == TARGET and size > 0:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + len(MAGIC))
    return out


def disassemble(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn", f.name],
                           check=True, capture_output=True, text=True)
    return r.stdout.splitlines()


def _regs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _lds_data_regs(op, ops):
    """VGPRs an LDS instruction reads as data (not the address)."""
    if op.startswith(("ds_bpermute", "ds_permute")):
        return _regs(ops[2]) if len(ops) > 2 else set()
    if op.startswith("ds_swizzle"):  # ds_swizzle_b32 vdst, vsrc offset:...
        return _regs(ops[1]) if len(ops) > 1 else set()
    if op.startswith(("ds_read", "ds_load", "ds_consume", "ds_append", "ds_nop")):
        return set()
    # stores / atomics: every operand after the address
    return set().union(*[_regs(o) for o in ops[1:]]) if len(ops) > 1 else set()


def scan(lines, min_states=MIN_STATES):
    """[(function, pk instruction, lds instruction, wait states)] hazards."""
    found, fn, win = [], None, []
    for raw in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:", raw)
        if m:
            fn, win = m.group(1), []
            continue
        s = raw.split("//")[0].strip()
        if not s or s.endswith(":"):
            continue
        op, _, rest = s.partition(" ")
        ops = [o.strip().split()[0] for o in re.split(r",\s*", rest.strip()) if o.strip()] if rest.strip() else []
        if op.startswith("ds_"):
            data = _lds_data_regs(op, ops)
            states = 0
            limit = None if op.startswith(CROSS_LANE) else min_states
            for pop, pops, ps in reversed(win):
                if (limit is not None and states >= limit) or not data:
                    break
                written = _regs(pops[0]) if pops and pop.startswith("v_") else set()
                if pop.startswith("v_pk_") and pop.endswith("_f32") and written & data:
                    found.append((fn, ps, s, states))
                data -= written
                states += int(pops[0], 0) + 1 if pop == "s_nop" else 1
        if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
            win = []
        else:
            win.append((op, ops, s))
    return found


def check(lib, min_states=MIN_STATES):
    hz = []
    for co in code_objects(lib):
        hz += scan(disassemble(co), min_states)
    return hz


def main():
    argv, args, ms = sys.argv[1:], [], MIN_STATES
    i = 0
    while i < len(argv):
        if argv[i] == "--strict":
            ms = None
        elif argv[i] == "--min-states":
            if i + 1 >= len(argv):
                sys.exit("--min-states needs a value")
            ms = int(argv[i + 1])
            i += 2
            continue
        if not argv[i].startswith("--"):
            args.append(argv[i])
        i += 1
    lib = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "modular_rl_amd", "libmrl_hip.so")
    hz = check(lib, ms)
    by_fn = {}
    for fn, pk, ds, st in hz:
        by_fn.setdefault(fn, []).append((pk, ds, st))
    for fn, v in sorted(by_fn.items()):
        print(f"{fn}: {len(v)}")
        for pk, ds, st in v[: (None if "--all" in sys.argv else 2)]:
            print(f"    {pk}  ->  {ds}   ({st} wait states)")
    rule = "in the same basic block" if ms is None else f"under {ms} wait states (cross-lane: whole block)"
    print(f"{len(hz)} packed-f32 -> LDS data reads {rule} in {len(by_fn)} kernels")
    return 1 if hz else 0


if __name__ == "__main__":
    sys.exit(main())
