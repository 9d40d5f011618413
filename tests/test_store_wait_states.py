"""Invariant of the hand-written store paths (CPU, source-level).

A 16-byte vector store reads its data VGPRs a few cycles after issue, and the
compiler's hazard recognizer does not look inside inline asm: hipcc (ROCm 7.2,
gfx950) once overwrote the data registers of a buffer store with an SGPR
soffset in the very next VALU instruction and ~1 % of packets came out with the
new values ("A hazard the compiler misses").  So every inline-asm
store in the product kernels must carry its own wait states (`s_nop` >= 1)
inside the same asm statement.  This test fails on a new store path that
forgets them, before any GPU run.
"""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STORE = re.compile(r"(buffer|global|flat)_store_(dword|b)\w*")
ASM = re.compile(r'asm\s*(?:volatile)?\s*\(\s*((?:"(?:[^"\\]|\\.)*"\s*)+)', re.S)


def asm_bodies(text):
    for m in ASM.finditer(text):
        yield "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(1))), text[:m.start()].count("\n") + 1


def test_every_inline_asm_store_carries_wait_states():
    found = 0
    for path in glob.glob(os.path.join(ROOT, "neptun_amd", "csrc", "*")):
        if not path.endswith((".hip", ".h", ".cpp")):
            continue
        # string-literal macros spliced into asm (cache-policy suffixes) read as ""
        text = re.sub(r"\bWG_\w+_ASM\b", '""', open(path).read())
        for body, line in asm_bodies(text):
            instrs = [i.strip() for i in body.replace("\\n", "\n").replace("\\t", "").split("\n")
                      if i.strip()]
            for k, ins in enumerate(instrs):
                if STORE.match(ins) and "dwordx4" in ins:
                    found += 1
                    nxt = instrs[k + 1] if k + 1 < len(instrs) else ""
                    m = re.match(r"s_nop\s+(\d+)", nxt)
                    assert m and int(m.group(1)) >= 1, (
                        f"{os.path.relpath(path, ROOT)}:{line}: '{ins}' is not followed by "
                        "s_nop >= 1 in the same asm statement")
    assert found >= 2  # gstore16 and store16 in wg_aead.hip
