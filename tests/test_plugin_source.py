"""The Mitsuba plugin source (mitsuba_plugin/vrlAmdIntegrator.cpp) cannot be
compiled here (it needs the mitsuba-ALVRL headers and Boost); this checks the
part of it that can go stale silently: every libalvrl entry point and
constant it uses is declared in include/*.h, and every entry point is
exported by the built libalvrl.so."""
import ctypes as C
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_plugin_uses_declared_exports():
    src = (ROOT / "mitsuba_plugin" / "vrlAmdIntegrator.cpp").read_text()
    headers = (ROOT / "include" / "alvrl.h").read_text() + (ROOT / "include" / "alvrl_host.h").read_text()
    calls = set(re.findall(r"\b(alvrl_[a-z0-9_]+)\s*\(", src))
    assert len(calls) >= 10
    lib = C.CDLL(str(ROOT / "mitsuba-alvrl_amd" / "libalvrl.so"))
    for f in sorted(calls):
        assert re.search(r"ALVRL_API\s+[\w\s\*]+?\b%s\s*\(" % f, headers), f"{f} not declared"
        assert hasattr(lib, f), f"{f} not exported"
    for k in set(re.findall(r"\b(ALVRL_[A-Z0-9_]*[A-Z0-9])\b", src)):
        assert re.search(r"#define\s+%s\b|\b%s\s*=" % (k, k), headers), f"{k} not defined"
    types = set(re.findall(r"\b(alvrl_[a-z_]+)\b(?=\s*[\*&\s]\s*\w)", src)) - calls
    for t in types:
        assert re.search(r"\}\s*%s\s*;|typedef struct %s\b" % (t, t), headers), f"type {t} not declared"


def test_plugin_runs_no_reference_code():
    """The plugin includes Mitsuba's public headers and the library's, never a
    source of the reference integrator (its vrlTracer.h used to run records
    mode's VRL tracing on the product side): records mode traces the VRLs in
    the library (alvrl_scene_ext::tracer)."""
    src = (ROOT / "mitsuba_plugin" / "vrlAmdIntegrator.cpp").read_text()
    incs = re.findall(r'^\s*#\s*include\s*[<"]([^>"]+)[>"]', src, re.M)
    assert incs and all(i.startswith(("mitsuba/", "hip/", "alvrl")) or "/" not in i and "." not in i
                        for i in incs), incs
    assert "vrlTracer" not in "".join(incs)
    assert "e.tracer = &m_tdesc" in src


def test_plugin_compiles_against_mitsuba_declarations(tmp_path):
    """The plugin compiles against a mock of exactly the Mitsuba declarations
    it uses (tests/mitsuba_mock/: signatures as in the mitsuba-ALVRL headers,
    MTS_IMPLEMENT_CLASS_S and MTS_EXPORT_PLUGIN as in class.h:219-226 and
    cobject.h:99-107).  A missing unserialization constructor, an abstract
    class, a call that does not match Mitsuba's API or an override that
    hides a base virtual with another signature (-Werror=overloaded-virtual)
    fails here.  The object must define the plugin entry points and the
    unserializers of the integrator and its two resources."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    hip = pathlib.Path("/opt/rocm/include/hip/hip_runtime_api.h")
    if not gxx or not hip.exists():
        import pytest
        pytest.skip("needs g++ and the HIP headers")
    mock = ROOT / "tests" / "mitsuba_mock"
    obj = tmp_path / "vrl_plugin.o"
    cmd = [gxx, "-std=c++11", "-c", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror",
           "-Werror=overloaded-virtual", "-D__HIP_PLATFORM_AMD__", f"-I{mock / 'include'}",
           f"-I{ROOT / 'include'}", "-I/opt/rocm/include", str(ROOT / "mitsuba_plugin" / "vrlAmdIntegrator.cpp"),
           "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    syms = subprocess.run(["nm", "-C", str(obj)], capture_output=True, text=True).stdout
    for s in ("T CreateInstance", "T GetDescription", "__vrlAmdIntegrator_unSer", "__AmdVrlSet_unSer",
              "__AmdClusterInfo_unSer"):
        assert s in syms, s
