"""Static instruction counts of one kernel in a hipcc -save-temps assembly file, by loop depth (the
compiler's "Loop Depth=k" block comments) and instruction class — where the persistent loop's
instructions are, before any GPU run.
usage: python tools/isa_stats.py <file.s> <kernel-symbol-substring> [--blocks]"""
import collections
import re
import sys


def kernel_body(text: str, key: str) -> tuple[str, str]:
    names = re.findall(r"^([A-Za-z_$][\w.$]*):", text, re.M)
    cand = [n for n in names if key in n and not n.startswith(".")]
    if not cand:
        raise SystemExit(f"no kernel matching {key!r}")
    name = min(cand, key=len)
    i = text.index("\n" + name + ":") + 1
    j = text.index(".Lfunc_end", i)
    return name, text[i:j]


def is_inst(line: str) -> bool:
    return line.startswith("\t") and not line.startswith("\t.") and not line.startswith("\t;")


def main():
    path, key = sys.argv[1], sys.argv[2]
    name, body = kernel_body(open(path).read(), key)
    blocks = re.split(r"\n(?=\.LBB|; %bb)", body)
    by_depth = collections.defaultdict(collections.Counter)
    rows = []
    for b in blocks:
        m = re.search(r"Depth=(\d+)", b.split("\n\t", 1)[0] + "\n" + "\n".join(b.split("\n")[:3]))
        d = int(m.group(1)) if m else 0
        ins = [ln.split()[0] for ln in b.split("\n") if is_inst(ln)]
        for op in ins:
            cls = ("v_f64" if op.startswith("v_") and "f64" in op else
                   "v_mad64" if op.startswith("v_mad_u64") or op.startswith("v_mad_i64") else
                   "v_other" if op.startswith("v_") else
                   "s" if op.startswith("s_") else
                   "mem" if op.split("_")[0] in ("global", "buffer", "flat", "ds", "scratch") else "other")
            by_depth[d][cls] += 1
        head = b.split("\n", 1)[0][:40]
        rows.append((head, d, len(ins), sum(1 for op in ins if op.startswith("v_"))))
    print(name)
    for d in sorted(by_depth):
        c = by_depth[d]
        print(f"depth {d}: total {sum(c.values()):5d}  " + "  ".join(f"{k} {v}" for k, v in sorted(c.items())))
    if "--blocks" in sys.argv:
        for head, d, n, v in rows:
            print(f"{d} {n:4d} {v:4d}  {head}")


if __name__ == "__main__":
    main()
