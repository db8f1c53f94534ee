"""Inline-asm lint for the HIP sources: a block that writes SCC (scalar ALU ops such as
s_or_b64 / s_and_b32 / s_add_u32 / s_cmp_*) or VCC (an explicit vcc destination) must declare
the "scc" / "vcc" clobber.  Round 4: glut_sel (nqk_glut.h) lacked "scc", and a build that
scheduled an s_cselect after the block stored through a zero-size buffer descriptor
(profiles/r04_glut_unpacked_dropped.txt)."""
import glob
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "numpy-quant_amd", "csrc")
SCC_WRITERS = re.compile(r"\bs_(or|and|xor|andn2|orn2|nand|nor|xnor|add|addc|sub|subb|lshl|lshr|ashr|bfe|cmp\w*|"
                         r"min|max|abs|not|bcnt\w*|ff\w*|bitcmp\w*|cselect)\w*\b")
VCC_WRITE = re.compile(r"\bv_\w+\s+vcc\b")


def _asm_blocks(text):
    """Every asm(...) / asm volatile(...) statement of a source, up to its closing parenthesis
    (macro line continuations joined)."""
    text = text.replace("\\\n", "\n")
    for m in re.finditer(r"\basm\s*(volatile\s*)?\(", text):
        depth, i = 1, m.end()
        while depth and i < len(text):
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        yield text[m.start():i]


def _sections(blk):
    """The asm statement's template (its string literals joined) and its clobber section:
    the ':'-separated sections split outside string literals and nested parentheses."""
    body = blk[blk.index("(") + 1:-1]
    parts, cur, depth, instr, i = [], "", 0, False, 0
    while i < len(body):
        ch = body[i]
        if instr:
            cur += ch
            if ch == "\\":
                cur += body[i + 1]
                i += 1
            elif ch == '"':
                instr = False
        elif ch == '"':
            instr = True
            cur += ch
        elif ch in "([":
            depth += 1
            cur += ch
        elif ch in ")]":
            depth -= 1
            cur += ch
        elif ch == ":" and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
        i += 1
    parts.append(cur)
    code = " ".join(re.findall(r'"((?:[^"\\]|\\.)*)"', parts[0]))
    code = code.replace("\\n", " ").replace("\\t", " ")  # the template's escaped separators
    return code, (parts[3] if len(parts) > 3 else "")


def test_inline_asm_declares_scc_and_vcc_clobbers():
    files = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
    assert files
    bad = []
    for f in files:
        for blk in _asm_blocks(open(f).read()):
            code, clobbers = _sections(blk)
            if SCC_WRITERS.search(code) and '"scc"' not in clobbers:
                bad.append((os.path.basename(f), "scc", code[:80]))
            if VCC_WRITE.search(code) and '"vcc"' not in clobbers:
                bad.append((os.path.basename(f), "vcc", code[:80]))
    assert not bad, bad


def test_lint_catches_a_missing_scc_clobber():
    blk = 'asm("v_cmp_le_u32 %[m], %[x], 5\\n\\ts_or_b64 %[s], %[s], %[m]" : [m] "=&s"(m), [s] "+s"(s) : [x] "v"(x) : "vcc")'
    (b,) = list(_asm_blocks(blk))
    code, clobbers = _sections(b)
    assert SCC_WRITERS.search(code) and '"vcc"' in clobbers
    assert '"scc"' not in clobbers
