"""Static instruction mix of kernels in a gfx950 assembly file (hipcc -S
--cuda-device-only): counts per opcode, VALU total, scratch ops.
    python tools/isa_mix.py file.s [substring ...]"""
import collections
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):\s*;", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        yield m.group(1), text[start:end]


def main():
    text = open(sys.argv[1]).read()
    want = sys.argv[2:]
    for name, body in kernels(text):
        if want and not any(w in name for w in want):
            continue
        ops = collections.Counter()
        for line in body.splitlines():
            t = line.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            ops[t[0]] += 1
        valu = sum(v for k, v in ops.items() if k.startswith("v_"))
        scratch = sum(v for k, v in ops.items() if "scratch" in k)
        print(f"{name}: VALU {valu}, scratch ops {scratch}, ds {sum(v for k, v in ops.items() if k.startswith('ds_'))}")
        print("   ", ", ".join(f"{k} {v}" for k, v in ops.most_common(24)))


if __name__ == "__main__":
    main()
