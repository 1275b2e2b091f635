"""Dev tool: per-kernel instruction mix of a hipcc -S listing (whole kernel and its hottest loop).

usage: python tools/asm_stats.py listing.s <kernel-substring> [...]
Loops are found from backward branches (s_cbranch_* / s_branch to an earlier label)."""
import collections
import re
import sys


def kernels(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+):\s*;", ln)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and ln.startswith(".Lfunc_end"):
            yield cur, body
            cur = None
            continue
        if cur:
            body.append(ln)


def klass(op):
    if "mfma" in op: return "mfma"
    if op.startswith("v_"):
        if any(x in op for x in ("mul_hi", "mul_lo", "mad_u64", "mad_i64")): return "valu_imul"
        if any(x in op for x in ("exp", "log", "rcp", "rsq", "sqrt")): return "valu_trans"
        return "valu"
    if op.startswith("ds_"): return "lds"
    if op.startswith(("buffer_", "global_", "flat_")): return "vmem"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith("s_"): return "salu"
    return "other"


def mix(body):
    c = collections.Counter()
    for ln in body:
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        c[klass(t.split()[0])] += 1
    return c


def hottest_loop(body):
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m: labels[m.group(1)] = i
    best = None
    for i, ln in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            seg = body[labels[m.group(2)]:i + 1]
            n = mix(seg)["mfma"]
            if best is None or n > best[0]: best = (n, seg)
    return best[1] if best else []


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().splitlines()
    for name, body in kernels(lines):
        if not any(s in name for s in sys.argv[2:]): continue
        print(name)
        print("  kernel:", dict(mix(body)))
        print("  loop  :", dict(mix(hottest_loop(body))))


def opcode_hist(listing, kname, top=45):
    lines = open(listing).read().splitlines()
    for name, body in kernels(lines):
        if kname in name:
            c = collections.Counter()
            for ln in hottest_loop(body):
                t = ln.strip()
                if t and not t.startswith((";", ".")) and not t.endswith(":"):
                    c[t.split()[0]] += 1
            return c.most_common(top)
