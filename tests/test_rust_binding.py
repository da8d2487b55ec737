"""The Rust crates under rust/ (rrte-hip-sys, rrte-renderer-hip) and the reference patches, checked
mechanically.  There is no cargo here, so they cannot be compiled; instead:

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
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rrte_hip.h"


SYS_LIB = ROOT / "rust" / "rrte-hip-sys" / "src" / "lib.rs"


def _rust_block():
    """rust/rrte-hip-sys/src/lib.rs without comments (the crate's FFI declarations)."""
    return re.sub(r"//[^\n]*", "", SYS_LIB.read_text())


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


def _rust_ffi_calls(text):
    """(name, argument count) of every `rrte_hip_*(...)` call in Rust source (parentheses balanced)."""
    out = []
    for m in re.finditer(r"\b(rrte_hip_\w+)\(", text):
        depth, i = 1, m.end()
        while depth and i < len(text):
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        inner = text[m.end():i - 1].strip()
        out.append((m.group(1), 0 if not inner else len(_split_top(inner))))
    return out


def test_safe_wrappers_call_the_ffi_with_the_declared_arity():
    """Every FFI call in the safe wrapper and the backend crate passes as many arguments as the header
    declares (no cargo here: a wrapper left behind by a signature change would not be compiled)."""
    hf = header_functions()
    files = [ROOT / "rust" / "rrte-hip-sys" / "src" / "safe.rs", ROOT / "rust" / "rrte-renderer-hip" / "src" / "lib.rs"]
    calls = []
    for f in files:
        t = _strip_comments(f.read_text())
        t = re.sub(r"pub fn rrte_hip_\w+\(", "pub fn X(", t)  # (declarations are checked above)
        calls += _rust_ffi_calls(t)
    assert len(calls) >= 10
    for name, n in calls:
        assert name in hf, name
        assert n == len(hf[name][1]), f"{name}: {n} arguments, header declares {len(hf[name][1])}"


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


# ------------------------------------------------------------------ the lowering
CPP = ROOT / "rrte_amd" / "cpp" / "rrte_renderer.cpp"
LOWER_RS = ROOT / "rust" / "rrte-renderer-hip" / "src" / "lower.rs"
SDF_RS = ROOT / "rust" / "rrte-renderer-hip" / "src" / "sdf.rs"


def _strip_comments(t):
    return re.sub(r"//[^\n]*", "", t)


def _norm(tok):
    """One argument, language-neutral: no casts, derefs, self., member underscores, f suffixes."""
    t = " ".join(tok.split())
    t = re.sub(r"\(float\)|\(double\)|\(uint32_t\)", "", t)
    t = re.sub(r"\s+as\s+(f32|f64|u32|i32)\b", "", t)
    t = t.replace("rrte_math::ZERO", "ZERO").replace("*", "").replace("self.", "").replace("?", "")
    t = re.sub(r"\b(\w+)_\b", r"\1", t)                     # albedo_ -> albedo (C++ member names)
    t = re.sub(r"(\d+\.\d*(?:e-?\d+)?)f\b", r"\1", t)      # 0.0f -> 0.0
    return t.replace(" ", "")


def _args(s):
    return [_norm(a) for a in _split_top(s)]


def _cpp_calls(fn_name_re, callee, text):
    """{kind constant: [args]} of `callee(KIND, ...)` inside C++ functions whose name matches."""
    out = {}
    for m in re.finditer(r"(\w+)::lower\([^)]*\) const \{", text):
        if not re.match(fn_name_re, m.group(1)):
            continue
        body = " ".join(text[m.end():m.end() + 400].split())  # the function's first call
        c = re.search(callee + r"\((RRTE_\w+),\s*(.*?)\);", body)
        if c:
            out[c.group(1)] = c.group(2)
    return out


def _braced(s):
    """`{a, b}` (C++ init list) or `&[a, b]` (Rust slice) -> inner text."""
    s = s.strip()
    m = re.match(r"&?[\[{](.*)[\]}]$", s, re.S)
    return m.group(1) if m else s


def test_prim_lowering_matches_the_cpp_mirror():
    """Every SceneObject: the same kind constant and the same p[] values in the same order as the
    C++ mirror's `X::lower` (which the GPU suite renders against the oracle)."""
    cpp = _strip_comments(CPP.read_text())
    want = {}
    for cls in ("Sphere", "Plane", "Triangle", "Cube", "Cylinder", "Cone", "Capsule"):
        m = re.search(cls + r"::lower\(Lowering&\) const \{(.*?)\n\}", cpp, re.S)
        body = " ".join(m.group(1).split())
        c = re.search(r"prim\((RRTE_PRIM_\w+),\s*\{(.*?)\}\)", body)
        want[c.group(1)] = _args(c.group(2))
    rs = " ".join(_strip_comments(LOWER_RS.read_text()).split())
    got = {}
    for kind, args in re.findall(r"prim\(\s*(RRTE_PRIM_(?:SPHERE|PLANE|TRIANGLE|CUBE|CYLINDER|CONE|CAPSULE)),\s*&\[(.*?)\],\s*t,?\s*\)", rs):
        got[kind] = _args(args)
    assert set(got) == set(want), (set(want) - set(got), set(got) - set(want))
    for kind in want:
        assert got[kind] == want[kind], (kind, got[kind], want[kind])
    # the transform columns: same fields in the same order
    c_trs = re.search(r"fill\(r\.trs, \{(.*?)\}\);", " ".join(cpp.split())).group(1)
    r_trs = re.search(r"r\.trs = \[(.*?)\];", rs).group(1)
    assert _args(c_trs) == _args(r_trs)


def test_sdf_object_lowering_matches_the_cpp_mirror():
    """SDFObject: the bound inflation and every march field the C++ lowering assigns."""
    cpp = " ".join(_strip_comments(CPP.read_text()).split())
    sdf = " ".join(_strip_comments(SDF_RS.read_text()).split())
    rs = " ".join(_strip_comments(LOWER_RS.read_text()).split())
    assert "const double r = b.r * 1.001 + 1e-3;" in cpp and "let r = b.r * 1.001 + 1e-3;" in sdf
    body = re.search(r"rrte_prim SDFObject::lower\(Lowering& lw\) const \{(.*?)return p; \}", cpp).group(1)
    cf = set(re.findall(r"\bp\.(sdf_\w+) =", body))
    rf = set(re.findall(r"\bp\.(sdf_\w+) =", rs))
    assert cf == rf == {"sdf_first", "sdf_count", "sdf_max_steps", "sdf_step_scale", "sdf_hit_eps"}
    assert "RRTE_PRIM_SDF" in rs
    # default march parameters and the deformer step scale
    assert "128, None, 1e-4" in sdf and "if sdf.has_deformer() { 0.6 } else { 1.0 }" in sdf
    assert "sdf->has_deformer() ? 0.6f : 1.0f" in cpp


def _cpp_defaults(cpp, fn):
    """Default arguments of a C++ helper signature: [(name, default or None)]."""
    sig = re.search(fn + r"\((.*?)\)\s*\{", " ".join(cpp.split())).group(1)
    out = []
    for a in _split_top(sig):
        name = a.split("=")[0].split()[-1]
        out.append((name, _norm(a.split("=", 1)[1]) if "=" in a else None))
    return out


def test_light_and_material_lowering_match_the_cpp_mirror():
    cpp = _strip_comments(CPP.read_text())
    rs = " ".join(_strip_comments(LOWER_RS.read_text()).split())
    lights = _cpp_calls(r".*Light$", "light_struct", cpp)
    defaults = _cpp_defaults(cpp, "rrte_light light_struct")
    got = dict(re.findall(r"light_struct\(\s*(RRTE_LIGHT_\w+),\s*(.*?)\)\s*(?:,\s*GpuLight|\}|$)", rs))
    assert set(lights) == set(got) == {"RRTE_LIGHT_POINT", "RRTE_LIGHT_DIRECTIONAL", "RRTE_LIGHT_SPOT",
                                       "RRTE_LIGHT_AMBIENT"}
    for kind, args in lights.items():
        a = _args(args)
        a += [d for _, d in defaults[1 + len(a):]]  # the C++ call's omitted arguments: their defaults
        assert _args(got[kind]) == a, (kind, _args(got[kind]), a)
    mats = _cpp_calls(r".*Material$", "material_struct", cpp)
    mgot = dict(re.findall(r"material_struct\((RRTE_MAT_\w+),\s*([^)]*)\)", rs))
    assert set(mats) == set(mgot) == {"RRTE_MAT_LAMBERTIAN", "RRTE_MAT_METAL", "RRTE_MAT_DIELECTRIC",
                                      "RRTE_MAT_EMISSIVE"}
    for kind, args in mats.items():
        assert _args(mgot[kind]) == _args(args), (kind, mgot[kind], args)
    # the helpers fill the same record fields
    for helper, var in (("light_struct", "l"), ("material_struct", "m")):
        cb = re.search(helper + r"\(.*?\)\s*\{(.*?)\n\}", cpp, re.S).group(1)
        rb = re.search(helper + r"\(.*?\)\s*->\s*\w+\s*\{(.*?)\}", rs).group(1)
        cf = set(re.findall(r"\b" + var + r"\.(\w+) =", cb)) | set(re.findall(r"fill\(" + var + r"\.(\w+),", cb))
        rf = set(re.findall(r"\b" + var + r"\.(\w+) =", rb))
        assert cf == rf, (helper, cf ^ rf)


def test_camera_and_config_lowering_match_the_cpp_mirror():
    cpp = " ".join(_strip_comments(CPP.read_text()).split())
    rs = " ".join(_strip_comments(LOWER_RS.read_text()).split())
    cb = re.search(r"rrte_camera Camera::lower\(\) const \{(.*?)return c; \}", cpp).group(1)
    rb = re.search(r"pub fn lower_camera\(.*?\{(.*?)\bc \}", rs).group(1)
    cf = set(re.findall(r"\bc\.(\w+) =", cb)) | set(re.findall(r"fill\(c\.(\w+),", cb))
    rf = set(re.findall(r"\bc\.(\w+) =", rb))
    assert cf == rf, cf ^ rf
    cb = re.search(r"rrte_render_params RaytracerConfig::lower\(\) const \{(.*?)return p; \}", cpp).group(1)
    rb = re.search(r"pub fn lower_config\(.*?\{(.*?)\bp \}", rs).group(1)
    cf = set(re.findall(r"\bp\.(\w+) =", cb)) | set(re.findall(r"fill\(p\.(\w+),", cb))
    rf = set(re.findall(r"\bp\.(\w+) =", rb))
    assert cf == rf, cf ^ rf


def _positional(args, params):
    """Arguments with the function's parameter names replaced by their positions ($0, $1, ...)."""
    out = []
    for a in args:
        for i, n in enumerate(params):
            a = re.sub(r"\b" + re.escape(n) + r"\b", f"${i}", a)
        out.append(a)
    return out


def test_sdf_builders_match_the_cpp_mirror():
    """The build-defined SDF surface (README.md:303-328, 496-510): every leaf builder emits the same
    node op and parameters, every deformer the same op, floats and integer arguments (parameters
    compared by position: the Rust names follow Rust conventions)."""
    cpp = " ".join(_strip_comments(CPP.read_text()).split())
    rs = " ".join(_strip_comments(SDF_RS.read_text()).split())

    def cparams(sig):
        return [a.split()[-1] for a in _split_top(sig)]

    def rparams(sig):
        return [a.split(":")[0].strip() for a in _split_top(sig)]

    leaves = ("sphere", "box", "cylinder", "prism", "torus", "tube", "ring", "cone", "capsule", "ellipsoid")
    for name in leaves:
        c = re.search(r"SDFRef sdf_" + name + r"\((.*?)\) \{.*?make_shared<Leaf>\((RRTE_SDF_\w+), c, std::vector<float>\{(.*?)\},", cpp)
        r = re.search(r"pub fn sdf_" + name + r"\((.*?)\) -> SdfRef \{.*?Leaf \{ op: (RRTE_SDF_\w+), c, f: vec!\[(.*?)\],", rs)
        assert c and r, name
        assert c.group(2) == r.group(2), name
        a, b = _positional(_args(c.group(3)), cparams(c.group(1))), _positional(_args(r.group(3)), rparams(r.group(1)))
        assert a == b, (name, a, b)
    for name in ("twist", "bend", "taper", "noise", "wave"):
        c = re.search(r"DeformerRef " + name + r"\((.*?)\) \{.*?node\((RRTE_SDF_\w+), \{(.*?)\}, \{(.*?)\}\)", cpp)
        r = re.search(r"pub fn " + name + r"\((.*?)\)\s*-> Result<DeformerRef, SdfError> \{.*?node\((RRTE_SDF_\w+), &\[(.*?)\], &\[(.*?)\]\)", rs)
        assert c and r, name
        assert c.group(2) == r.group(2), name
        cp, rp = cparams(c.group(1)), rparams(r.group(1))
        for k in (3, 4):
            a, b = _positional(_args(c.group(k)), cp), _positional(_args(r.group(k)), rp)
            assert a == b, (name, a, b)


# ------------------------------------------------------------ the reference patches
PATCHES = ROOT / "rust" / "patches"
REFERENCE = Path("/root/reference")


def test_patches_hook_every_reference_type():
    p1 = (PATCHES / "0001-rrte-renderer-gpu-desc.patch").read_text()
    for cls in ("Sphere", "Plane", "Triangle", "Cube", "Cylinder", "Cone", "Capsule"):
        assert re.search(r"impl SceneObject for " + cls + r" \{\n\+    fn gpu_desc", p1), cls
    for cls in ("DirectionalLight", "PointLight", "SpotLight", "AmbientLight"):
        assert re.search(r"impl Light for " + cls + r" \{\n\+    fn gpu_desc", p1), cls
    for cls in ("LambertianMaterial", "MetalMaterial", "DielectricMaterial", "EmissiveMaterial"):
        assert re.search(r"impl Material for " + cls + r" \{\n\+    fn gpu_desc", p1), cls
    assert "+pub trait RenderBackend" in p1 and "+    pub fn set_backend" in p1
    # the fast boundary: a defaulted RenderBackend::render_into and Raytracer::render_into,
    # Raytracer::render's signature unchanged
    assert "+    fn render_into(&self, objects: &[Arc<dyn SceneObject>]" in p1
    assert "+    pub fn render_into(" in p1 and "+        out: &mut Vec<u8>," in p1
    assert "-    ) -> Vec<u8> {" not in p1
    p2 = (PATCHES / "0002-rrte-core-hip-backend.patch").read_text()
    # Engine::render_frame renders into its own reused frame_buffer (engine.rs:82,293), not a fresh Vec
    assert ("+                raytracer.render_into(self.scene.get_objects(), self.scene.get_lights(),\n"
            "+                                      self.scene.get_materials(), &self.camera, &mut self.frame_buffer);") in p2
    assert "self.frame_buffer = raytracer.render(" not in p2.replace("-                self.frame_buffer", "")
    assert "rrte_renderer_hip::HipBackend::new" in p2


def test_backend_keeps_the_engine_buffer_pinned():
    """HipBackend::render_into (rust/rrte-renderer-hip) goes through Context::render_engine_frame, which
    pins the engine's buffer once and re-pins only a buffer that moved; the context's own frame buffer
    is page-aligned whole pages (no page shared with another registration)."""
    lib = (ROOT / "rust" / "rrte-renderer-hip" / "src" / "lib.rs").read_text()
    safe = (ROOT / "rust" / "rrte-hip-sys" / "src" / "safe.rs").read_text()
    assert "fn render_into(&self" in lib and "ctx.render_engine_frame(&scene, &params, out)" in lib
    body = safe[safe.index("pub fn render_engine_frame"):safe.index("pub fn unpin_engine_frame")]
    assert body.index("self.unpin_engine_frame()?") < body.index("out.resize(need, 0)")  # unpin before a move
    assert "rrte_hip_host_register(self.ctx, out.as_mut_ptr()" in body and "self.unpinnable = addr" in body
    assert "Layout::from_size_align(size, PAGE)" in safe and "& !(PAGE - 1)" in safe


@pytest.mark.skipif(not REFERENCE.exists(), reason="the reference checkout is not on this machine")
def test_patches_apply_and_are_current(tmp_path):
    """The committed patches apply to the reference snapshot and equal what tools/make_rust_patches.py
    generates from it."""
    import shutil
    work = tmp_path / "ref"
    work.mkdir()
    shutil.copy(REFERENCE / "Cargo.toml", work / "Cargo.toml")
    shutil.copytree(REFERENCE / "crates", work / "crates")
    for p in sorted(PATCHES.glob("*.patch")):
        r = subprocess.run(["patch", "-p1", "--forward", "-i", str(p)], cwd=work, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    assert (work / "crates/rrte-renderer/src/gpu_desc.rs").exists()
    gen = tmp_path / "gen"
    env = dict(__import__("os").environ, RRTE_REFERENCE=str(REFERENCE))
    code = (f"import sys; sys.path.insert(0, {str(ROOT / 'tools')!r}); import make_rust_patches as m; "
            f"from pathlib import Path; m.OUT = Path({str(gen)!r}); m.main()")
    subprocess.run([sys.executable, "-c", code], check=True, env=env, capture_output=True)
    for p in sorted(PATCHES.glob("*.patch")):
        assert (gen / p.name).read_text() == p.read_text(), f"{p.name} is stale: rerun tools/make_rust_patches.py"


def test_lowering_checker_catches_a_swapped_argument(monkeypatch, tmp_path):
    """The checker itself: a Rust lowering that swaps a cylinder's radius and height must fail."""
    bad = LOWER_RS.read_text().replace("prim(RRTE_PRIM_CYLINDER, &[center.x, center.y, center.z, *radius, *height], t)",
                                       "prim(RRTE_PRIM_CYLINDER, &[center.x, center.y, center.z, *height, *radius], t)")
    assert bad != LOWER_RS.read_text()
    f = tmp_path / "lower.rs"
    f.write_text(bad)
    monkeypatch.setattr(sys.modules[__name__], "LOWER_RS", f)
    with pytest.raises(AssertionError):
        test_prim_lowering_matches_the_cpp_mirror()
