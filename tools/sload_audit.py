"""List scalar (s_load) reads that are NOT kernarg reads, per kernel, from hipcc -S output.

A load at a wave-uniform address compiles to s_load_*, which goes through the scalar data
cache; that cache did not see vector stores made by an earlier launch of the same stream
(k_expand read stale leaf records this way, round 2).  Every s_load here must read data
that no earlier kernel of the engine rewrites (kernargs, weights, tables), or be turned
into a vector load.  Usage: python tools/sload_audit.py file.s [...]"""
import re
import sys

for path in sys.argv[1:]:
    lines = open(path).read().splitlines()
    kern = None
    body = []
    meta = {}

    def flush():
        if kern is None:
            return
        # user SGPR layout: private segment buffer (4), dispatch ptr (2), queue ptr (2), kernarg ptr (2)
        base = 0
        base += 4 if meta.get("private_segment_buffer") else 0
        base += 2 if meta.get("dispatch_ptr") else 0
        base += 2 if meta.get("queue_ptr") else 0
        karg = "s[%d:%d]" % (base, base + 1)
        disp = "s[%d:%d]" % (base - 4, base - 3) if meta.get("dispatch_ptr") and meta.get("queue_ptr") else \
            ("s[%d:%d]" % (base - 2, base - 1) if meta.get("dispatch_ptr") else None)
        # registers that hold pointers loaded straight from kernarg stay suspicious: report all
        bad = [l.strip() for l in body if re.search(r"\bs_load_", l) and karg not in l and (disp is None or disp not in l)]
        if bad:
            print("%s: %d non-kernarg s_load" % (kern, len(bad)))
            for b in bad[:6]:
                print("    " + b)

    for l in lines:
        m = re.match(r"^(_Z\w+):", l)
        if m:
            flush()
            kern, body, meta = m.group(1), [], {}
            continue
        m = re.search(r"\.amdhsa_user_sgpr_(\w+)\s+(\d)", l)
        if m and kern:
            meta[m.group(1)] = int(m.group(2))
            continue
        if kern:
            body.append(l)
    flush()
