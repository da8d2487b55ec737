"""The Rust `-sys` binding in INTEGRATION.md §1, checked mechanically against include/rrte_hip.h
(VERDICT r02 #9).  There is no cargo here, so the block cannot be compiled; instead:

* every `#[repr(C)]` struct: field names and order equal the header's, and the repr(C) layout the
  Rust types imply (offsets, size) equals offsetof/sizeof from a C program compiled with the header;
* every `pub const` equals the header's #define / enum value;
* every `extern "C"` function: the header declares it, with the same argument count and C types
  (canonicalised: uint32_t = u32, int = c_int = i32, T* = *mut T, const T* = *const T, arrays decay),
  and every header entry point is bound.

The real caller this protects is crates/rrte-renderer/src/raytracer.rs:35-51 via
crates/rrte-core/src/engine.rs:280-312 (a struct-layout drift would corrupt every frame silently)."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rrte_hip.h"


def _rust_block():
    text = (ROOT / "INTEGRATION.md").read_text()
    blocks = re.findall(r"```rust\n(.*?)```", text, re.S)
    lib = [b for b in blocks if "crates/rrte-hip-sys/src/lib.rs" in b]
    assert len(lib) == 1, "INTEGRATION.md must hold exactly one rrte-hip-sys lib.rs block"
    return re.sub(r"//[^\n]*", "", lib[0])


def _split_top(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "[(<":
            depth += 1
        elif ch in "])>":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out if x.strip()]


def rust_structs(src):
    out = {}
    for name, body in re.findall(r"pub struct (\w+)\s*\{(.*?)\}", src, re.S):
        fields = []
        for f in _split_top(body):
            m = re.match(r"(?:pub\s+)?(\w+)\s*:\s*(.+)$", f, re.S)
            assert m, f
            fields.append((m.group(1), " ".join(m.group(2).split())))
        out[name] = fields
    return out


_PRIM = {"u8": (1, 1), "i8": (1, 1), "u32": (4, 4), "i32": (4, 4), "f32": (4, 4), "u64": (8, 8), "i64": (8, 8),
         "f64": (8, 8), "usize": (8, 8), "c_int": (4, 4), "c_char": (1, 1)}


def rust_layout(structs):
    """repr(C): each field at the next multiple of its alignment, size rounded up to the struct's."""
    memo = {}

    def ty(t):
        t = t.strip()
        if t.startswith("*"):
            return 8, 8
        m = re.match(r"\[(.+);\s*(\d+)\]$", t)
        if m:
            sz, al = ty(m.group(1))
            return sz * int(m.group(2)), al
        if t in _PRIM:
            return _PRIM[t]
        return lay(t)[0:2]

    def lay(name):
        if name in memo:
            return memo[name]
        off, al, offs = 0, 1, []
        for fname, t in structs[name]:
            sz, a = ty(t)
            off = (off + a - 1) // a * a
            offs.append((fname, off))
            off += sz
            al = max(al, a)
        size = (off + al - 1) // al * al
        memo[name] = (size, al, offs)
        return memo[name]

    return {n: lay(n) for n in structs}


def header_structs():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef struct \w+ \{(.*?)\}\s*(\w+);", text, re.S):
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            # "float a, b;"  "const rrte_prim* prims"  "uint32_t i[3]"
            parts = decl.split(",")
            first = re.match(r"(.*?)([\w]+)\s*(\[[^\]]*\])?$", parts[0].strip(), re.S)
            names.append(first.group(2))
            for p in parts[1:]:
                names.append(re.match(r"\s*\**\s*(\w+)", p).group(1))
        out[name] = names
    return out


def c_offsets(structs, tmp_path):
    """offsetof / sizeof of every Rust-named field, from a C program compiled with the header."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for name, fields in structs.items():
        if name == "rrte_ctx":
            continue
        lines.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for f, _ in fields:
            lines.append(f'printf("{name}.{f} %zu\\n", offsetof({name}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-o", str(exe), str(src)], check=True)
    res = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        k, v = line.split()
        res[k] = int(v)
    return res


def test_struct_fields_and_layout_match_header(tmp_path):
    src = _rust_block()
    rs = rust_structs(src)
    hs = header_structs()
    expected = {"rrte_prim": 192, "rrte_material": 32, "rrte_light": 80, "rrte_sdf_node": 64, "rrte_camera": 80,
                "rrte_render_params": 64, "rrte_mesh_vertex": 24}
    for name in set(hs) | set(expected):
        assert name in rs, f"INTEGRATION.md lacks a Rust mirror of {name}"
    for name, fields in rs.items():
        if name == "rrte_ctx":
            continue
        assert name in hs, f"{name} is not a header struct"
        assert [f for f, _ in fields] == hs[name], f"{name}: field names/order differ from the header"
    lay = rust_layout({k: v for k, v in rs.items() if k != "rrte_ctx"})
    c = c_offsets(rs, tmp_path)
    for name, (size, _, offs) in lay.items():
        assert size == c[name], f"{name}: Rust repr(C) size {size} != C sizeof {c[name]}"
        for f, off in offs:
            assert off == c[f"{name}.{f}"], f"{name}.{f}: Rust offset {off} != C offsetof {c[name + '.' + f]}"
        if name in expected:
            assert size == expected[name]


def _c_consts():
    text = HEADER.read_text()
    vals = {k: int(v) for k, v in re.findall(r"#define (RRTE_\w+) (\d+)u?\b", text)}
    for body in re.findall(r"typedef enum \w+ \{(.*?)\}", text, re.S):
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        for k, v in re.findall(r"(RRTE_\w+)\s*=\s*(\d+)", body):
            vals[k] = int(v)
    return vals


def test_constants_match_header():
    consts = dict((k, int(v)) for k, v in re.findall(r"pub const (RRTE_\w+): \w+ = (\d+);", _rust_block()))
    assert len(consts) >= 10
    cv = _c_consts()
    for k, v in consts.items():
        assert k in cv, k
        assert cv[k] == v, (k, v, cv[k])


_RUST_T = {"u32": "u32", "i32": "i32", "c_int": "i32", "f32": "f32", "u64": "u64", "f64": "f64", "usize": "usize",
           "u8": "u8", "c_char": "i8", "c_void": "void", "rrte_status": "i32"}
_C_T = {"uint32_t": "u32", "int32_t": "i32", "int": "i32", "float": "f32", "uint64_t": "u64", "double": "f64",
        "size_t": "usize", "uint8_t": "u8", "char": "i8", "void": "void", "rrte_status": "i32"}


def _rust_type(t):
    t = " ".join(t.split())
    m = re.match(r"\*(const|mut) (.+)$", t)
    if m:
        return ("const*" if m.group(1) == "const" else "*") + _rust_type(m.group(2))
    return _RUST_T.get(t, t)


def _c_param(p):
    p = " ".join(p.split())
    arr = re.search(r"\[[^\]]*\]$", p)
    p = re.sub(r"\[[^\]]*\]$", "", p).strip()
    const = p.startswith("const ")
    p = p[6:] if const else p
    m = re.match(r"(\w+)\s*(\**)\s*(\w*)$", p)
    base, stars = m.group(1), m.group(2)
    stars += "*" if arr else ""
    base = _C_T.get(base, base)
    if not stars:
        return base
    inner = base
    for k in range(len(stars)):
        inner = ("const*" if const and k == 0 else "*") + inner
    return inner


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^(rrte_status|uint32_t|void|const char\*)\s+(rrte_hip_\w+)\((.*?)\);", text,
                                      re.S | re.M):
        params = [] if args.strip() in ("", "void") else [_c_param(a) for a in _split_top(args)]
        r = {"rrte_status": "i32", "uint32_t": "u32", "void": "void", "const char*": "const*i8"}[ret]
        out[name] = (r, params)
    return out


def rust_functions():
    block = re.search(r'extern "C" \{(.*?)\n\}', _rust_block(), re.S).group(1)
    out = {}
    for name, args, ret in re.findall(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, re.S):
        params = [_rust_type(a.split(":", 1)[1]) for a in _split_top(args)]
        out[name] = (_rust_type(ret) if ret else "void", params)
    return out


def test_extern_functions_match_header():
    hf, rf = header_functions(), rust_functions()
    assert len(hf) >= 20
    assert set(rf) == set(hf), f"bound but not declared: {set(rf) - set(hf)}; declared but not bound: {set(hf) - set(rf)}"
    for name, (ret, params) in hf.items():
        assert rf[name] == (ret, params), f"{name}: Rust {rf[name]} != C {(ret, params)}"


def test_python_bindings_cover_the_header():
    from rrte_amd import abi
    assert set(abi.EXPORTS) == set(header_functions())


@pytest.mark.parametrize("mutate", ["swap", "width"])
def test_checker_catches_a_layout_drift(mutate, tmp_path):
    """The checker itself: a swapped field or a wrong field type must be caught."""
    rs = rust_structs(_rust_block())
    fields = list(rs["rrte_render_params"])
    if mutate == "swap":
        fields[0], fields[1] = fields[1], fields[0]
        assert [f for f, _ in fields] != header_structs()["rrte_render_params"]
    else:
        fields[-1] = (fields[-1][0], "u64")
        lay = rust_layout({"rrte_render_params": fields})
        c = c_offsets({"rrte_render_params": fields}, tmp_path)
        assert lay["rrte_render_params"][0] != c["rrte_render_params"]
