"""LDS-ordering audit of the device assembly (hipcc --cuda-device-only -S).

For every kernel, a dataflow pass over its basic blocks tracks the LDS-counter (lgkmcnt)
and vector-memory-counter (vmcnt) operations still in flight at each instruction, oldest
first, and reports every `s_barrier` reached while one of them is

  * an LDS write (ds_write*, ds_store*, ds atomics): another wave may read the old value
    after the barrier -- a race that only shows when the waves' timing shifts (e.g. when
    another queue's kernels share the CU);
  * a global_load_lds / buffer_load ... lds transfer: the data may not have landed.
    Kernels that deliberately keep the NEXT buffer's transfer in flight across a barrier
    show up here too; each such report is checked by hand against the buffer it targets.

On gfx950 the compiler does not insert waits before a bare s_barrier (the hardware has
back-off barriers), so `__builtin_amdgcn_s_barrier()` without a preceding wait is exactly
the case this looks for.  usage: isa_audit.py FILE.s [...]
"""
import re
import sys

LDS_WRITE = re.compile(r"^ds_(write|store|add|sub|inc|dec|min|max|and|or|xor|mskor|cmpst|cmpswap|wrxchg|condxchg|append|consume)")
LDS_OP = re.compile(r"^ds_")
SMEM = re.compile(r"^s_(load|buffer_load|store|memtime|memrealtime|dcache|atc_probe)")
VMEM_LDS = re.compile(r"^(global_load_lds|buffer_load\S*)\b")
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
BRANCH = re.compile(r"^s_(branch|cbranch_\w+)\s+(\S+)")
WAIT = re.compile(r"^s_waitcnt\b(.*)")
CAP = 64


def parse_wait(args):
    vm = lgkm = None
    m = re.search(r"vmcnt\((\d+)\)", args)
    if m:
        vm = int(m.group(1))
    m = re.search(r"lgkmcnt\((\d+)\)", args)
    if m:
        lgkm = int(m.group(1))
    if re.fullmatch(r"\s*(0x)?0\s*", args):  # s_waitcnt 0
        vm = lgkm = 0
    return vm, lgkm


def merge(a, b):
    """Outstanding-op lists (oldest first, True = tracked kind); align on the newest."""
    n = max(len(a), len(b))
    pa = (False,) * (n - len(a)) + a
    pb = (False,) * (n - len(b)) + b
    return tuple(x or y for x, y in zip(pa, pb))[-CAP:]


def kernels(lines):
    name, body = None, []
    for ln in lines:
        m = re.match(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$", ln)
        if m and not m.group(1).startswith(".L"):
            if name and body:
                yield name, body
            name, body = m.group(1), []
            continue
        if name is not None:
            body.append(ln)
            if ln.strip().startswith("s_endpgm"):
                yield name, body
                name, body = None, []


def audit(name, body):
    # basic blocks: split at .L labels and after branches
    blocks, labels, cur = [], {}, []
    for ln in body:
        s = ln.split(";")[0].strip()
        if not s or s.startswith("."):
            m = re.match(r"^(\.L\w+):", ln.strip())
            if m:
                if cur:
                    blocks.append(cur)
                cur = []
                labels[m.group(1)] = len(blocks)
            continue
        cur.append(s)
        if BRANCH.match(s) or s.startswith("s_endpgm") or s.startswith("s_setpc"):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    succ = []
    for i, b in enumerate(blocks):
        last = b[-1] if b else ""
        m = BRANCH.match(last)
        s = []
        if m:
            if m.group(2) in labels:
                s.append(labels[m.group(2)])
            if m.group(1) != "branch" and i + 1 < len(blocks):
                s.append(i + 1)
        elif not last.startswith("s_endpgm") and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    state_in = [None] * len(blocks)
    state_in[0] = ((), ())
    reports = {}
    work = [0]
    while work:
        i = work.pop()
        lg, vm = state_in[i]
        for j, ins in enumerate(blocks[i]):
            op = ins.split()[0]
            w = WAIT.match(ins)
            if w:
                v, l = parse_wait(w.group(1))
                if l is not None:
                    lg = lg[len(lg) - l:] if l < len(lg) else lg
                    if l == 0:
                        lg = ()
                if v is not None:
                    vm = vm[len(vm) - v:] if v < len(vm) else vm
                    if v == 0:
                        vm = ()
                continue
            if op == "s_barrier":
                if any(lg):
                    reports.setdefault((i, j, "LDS write in flight"), sum(lg))
                if any(vm):
                    reports.setdefault((i, j, "LDS DMA in flight"), sum(vm))
                continue
            if LDS_OP.match(op):
                lg = (lg + (bool(LDS_WRITE.match(op)),))[-CAP:]
            elif SMEM.match(op):
                lg = (lg + (False,))[-CAP:]
            elif VMEM.match(op):
                is_dma = op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in ins)
                vm = (vm + (is_dma,))[-CAP:]
        for k in succ[i]:
            new = (lg, vm) if state_in[k] is None else (merge(state_in[k][0], lg), merge(state_in[k][1], vm))
            if new != state_in[k]:
                state_in[k] = new
                work.append(k)
    return sorted(reports.items())


def main(paths):
    total = 0
    for p in paths:
        with open(p) as f:
            lines = f.read().splitlines()
        for name, body in kernels(lines):
            reps = audit(name, body)
            if not reps:
                continue
            kinds = {}
            for (_, _, kind), n in reps:
                kinds.setdefault(kind, []).append(n)
            desc = ", ".join(f"{k}: {len(v)} barrier(s), up to {max(v)} op(s)" for k, v in kinds.items())
            print(f"{p}: {name}: {desc}")
            total += sum(1 for (_, _, k), _ in reps if k == "LDS write in flight")
    print(f"barriers with an LDS write in flight: {total}")


if __name__ == "__main__":
    main(sys.argv[1:])
