#!/usr/bin/env python3
"""Prepare library sources for the host emulation build (tools_cpu/bdemu).

Extracts deap_amd/csrc/* and include/deapmi.h from a git revision (default:
cf1cf3a^, the last tree with the m = 4 bitset kernels) or from the working
tree ("worktree"), and rewrites the few constructs a host C++ compiler cannot
take:

  kernel<<<grid, block[, shm[, stream]]>>>(args);
      -> emu::launch(emu::cfg(grid, block, shm, stream), "kernel", [&]() { kernel(args); });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      -> emu::fence();
  asm volatile("v_writelane_b32 ..." : "+v"(o) : "s"(v), "i"(L));  -> emu_writelane(o, v, L);
  asm [volatile]("v_addc_co_u32_e64 ..." : "=v"(out), "=s"(c) : "v"(t), "v"(a), "s"(m));
      -> out = t + a + carry-in bit `lane` of m;
  extern __shared__ ... T name[];                        -> T* name = (T*)emu::dyn_lds();

The rewritten tree is build output (tools_cpu/bdemu/build/, git-ignored); no
source is copied into the repository.  Usage: prep.py REV OUTDIR
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FILES = ["common.hpp", "sort.hpp", "dominance.hpp", "bitdom.hpp", "transpose.hpp",
         "dominance.hip", "bitdom.hip", "nsga2.hip"]


def read(rev, path):
    if rev == "worktree":
        with open(os.path.join(REPO, path)) as f:
            return f.read()
    return subprocess.run(["git", "-C", REPO, "show", "%s:%s" % (rev, path)], check=True,
                          capture_output=True, text=True).stdout


def match_close(s, i, op, cl):
    """Index of the bracket closing s[i] == op."""
    depth = 0
    j = i
    while j < len(s):
        c = s[j]
        if c == op:
            depth += 1
        elif c == cl:
            depth -= 1
            if depth == 0:
                return j
        j += 1
    raise ValueError("unbalanced %s at %d" % (op, i))


def rewrite_launches(s):
    out = []
    pos = 0
    while True:
        i = s.find("<<<", pos)
        if i < 0:
            out.append(s[pos:])
            return "".join(out)
        # callee: identifier chars, '::' and balanced template arguments, backwards
        j = i
        while j > 0 and s[j - 1] == " ":
            j -= 1
        if s[j - 1] == ">":  # template arguments
            depth = 0
            k = j - 1
            while k >= 0:
                if s[k] == ">":
                    depth += 1
                elif s[k] == "<":
                    depth -= 1
                    if depth == 0:
                        break
                k -= 1
            j = k
        while j > 0 and (s[j - 1].isalnum() or s[j - 1] in "_:"):
            j -= 1
        callee = s[j:i].strip()
        e = s.find(">>>", i)
        cfg = s[i + 3:e]
        a = e + 3
        while s[a].isspace():
            a += 1
        assert s[a] == "(", "launch without arguments near %r" % s[j:a + 20]
        b = match_close(s, a, "(", ")")
        args = s[a + 1:b]
        name = re.sub(r"\s+", "", callee)
        out.append(s[pos:j])
        out.append('emu::launch(emu::cfg(%s), "%s", [&]() { %s(%s); })' % (cfg, name, callee, args))
        pos = b + 1


def rewrite(s):
    s = s.replace('asm volatile("s_waitcnt vmcnt(0)" ::: "memory");', "emu::fence();")
    s = re.sub(r'asm volatile\("v_writelane_b32 %0, %1, %2"\s*:\s*"\+v"\((\w+)\)\s*:\s*"s"\((\w+)\),\s*"i"\((\w+)\)\);',
               r"emu_writelane(\1, \2, \3);", s)
    s = re.sub(r'asm(?: volatile)?\("v_addc_co_u32_e64 %0, %1, %2, %3, %4"\s*:\s*"=v"\((\w+)\),\s*"=s"\((\w+)\)\s*'
               r':\s*"v"\((\w+)\),\s*"v"\((\w+)\),\s*"s"\((\w+)\)\);',
               r"\1 = \3 + \4 + (uint32_t)((\5 >> emu::lane()) & 1); \2 = 0;", s)
    s = re.sub(r"extern __shared__[^;\[]*?(\w+)\s+(\w+)\[\];", r"\1* \2 = (\1*)emu::dyn_lds();", s)
    if "asm" in re.sub(r"//.*", "", s).replace("emu::", ""):
        for ln in s.splitlines():
            if re.search(r"\basm\b", ln.split("//")[0]):
                raise SystemExit("prep: unhandled inline asm: " + ln.strip())
    s = register_lds(s)
    for pat, rep in CHECKS:
        s = s.replace(pat, rep)
    return rewrite_launches(s)


def register_lds(s):
    """Append EMU_LDS(name) after every __shared__ declaration: the runtime
    fills each registered array with a poison pattern before every workgroup
    (LDS content is undefined at workgroup start; the host's static storage
    would otherwise read as zeros or as the previous workgroup's values)."""
    def rep(mo):
        decl = mo.group(0)
        body = decl[len("__shared__"):-1]
        parts, depth, cur = [], 0, ""
        for ch in body:
            if ch in "[(":
                depth += 1
            elif ch in "])":
                depth -= 1
            if ch == "," and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        parts.append(cur)
        names = []
        for part in parts:
            head = part.split("[")[0]
            ids = re.findall(r"[A-Za-z_]\w*", head)
            names.append(ids[-1])
        return decl + "".join(" EMU_LDS(%s);" % n for n in names)
    return re.sub(r"(?m)(?<=^)[ \t]*__shared__[^;{}]*;", lambda mo: rep_ws(mo, rep), s)


def rep_ws(mo, rep):
    text = mo.group(0)
    ws = text[:len(text) - len(text.lstrip())]
    class M:
        def group(self, i):
            return text.lstrip()
    return ws + rep(M())


# index checks inside the 2-D LDS tables (ASan bounds a whole array, not its
# rows): the bucket search of bitdom.hpp and the prefix-set index k
CHECKS = [
    ("    const int b = x >> sh;\n    int j = sb[b];",
     "    const int b = x >> sh;\n    EMU_CHECK(b >= 0 && b + 1 < BD_BKN, \"bucket\", b);\n    int j = sb[b];"),
    ("        const int32_t y = sr[bd_rpad(j)];",
     "        EMU_CHECK(j >= 0 && j < BD_CW, \"sorted rank\", j);\n        const int32_t y = sr[bd_rpad(j)];"),
    ("        ++j;\n    }\n    return j;\n}",
     "        ++j;\n    }\n    EMU_CHECK(j >= 0 && j <= BD_CW, \"set index k\", j);\n    return j;\n}"),
]


def main():
    rev, out = sys.argv[1], sys.argv[2]
    src = os.path.join(out, "deap_amd", "csrc")
    inc = os.path.join(out, "include")
    os.makedirs(src, exist_ok=True)
    os.makedirs(inc, exist_ok=True)
    for f in FILES:
        try:
            text = read(rev, "deap_amd/csrc/" + f)
        except subprocess.CalledProcessError:
            continue  # a file this revision does not have
        with open(os.path.join(src, f), "w") as fh:
            fh.write(rewrite(text))
    with open(os.path.join(inc, "deapmi.h"), "w") as fh:
        fh.write(read(rev, "include/deapmi.h"))


if __name__ == "__main__":
    main()
