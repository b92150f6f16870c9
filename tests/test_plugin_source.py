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
