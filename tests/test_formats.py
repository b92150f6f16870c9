"""On-disk formats, no GPU needed: the vrlClusterInfo
stream against the byte layout of the reference's serialize()
(vrlIntegrator.cpp:66-101), the OpenEXR writer against an independent parse
of the file, mtsutil rms (src/utils/rms.cpp) against a numpy restatement, and
the dumpPass file name (integrator.cpp:361-378, vrlIntegrator.cpp:357-364)."""
import os
import re
import struct

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def _info():
    rng = np.random.default_rng(7)
    W, H, ns = 5, 3, 3
    slices = rng.integers(0, ns, W * H).astype(np.uint32)
    slices[4] = 0xFFFFFFFF                      # a pixel without a slice
    off = np.array([0, 2, 2, 5], np.uint32)     # an empty slice in the middle
    reps = np.array([9, 1, 4, 0, 7], np.uint32)
    w = rng.random(5).astype(np.float32)
    return {"slices": slices, "slice_off": off, "reps": reps, "weights": w,
            "global_reps": np.array([3], np.uint32), "global_weights": np.array([2.5], np.float32),
            "fb_reps": np.array([2, 8], np.uint32), "fb_weights": np.array([1.0, 0.5], np.float32)}


def _reference_stream(info):
    """vrlClusterInfo::serialize with Mitsuba's Stream on a little-endian host."""
    b = bytearray()
    ul = lambda n: b.extend(struct.pack("<Q", n))
    b += struct.pack("<Q", len(info["slices"])) + info["slices"].astype("<u4").tobytes()
    off = info["slice_off"]
    ns = len(off) - 1
    ul(ns)
    for s in range(ns):
        ul(int(off[s + 1] - off[s]))
        b += info["reps"][off[s]:off[s + 1]].astype("<u4").tobytes()
    ul(ns)
    for s in range(ns):
        ul(int(off[s + 1] - off[s]))
        b += info["weights"][off[s]:off[s + 1]].astype("<f4").tobytes()
    for k, t in (("global_reps", "<u4"), ("global_weights", "<f4"), ("fb_reps", "<u4"), ("fb_weights", "<f4")):
        ul(len(info[k]))
        b += info[k].astype(t).tobytes()
    return bytes(b)


def test_cluster_info_layout_and_roundtrip(alvrl, tmp_path):
    info = _info()
    p = str(tmp_path / "ci.bin")
    alvrl.write_cluster_info(p, info)
    assert open(p, "rb").read() == _reference_stream(info)
    back = alvrl.read_cluster_info(p)
    for k, v in info.items():
        assert np.array_equal(back[k].view(np.uint32), v.view(np.uint32)), k
    # the fall-back ids land in the id list (the reference's reader slip at :56-59 is fixed)
    assert back["fb_reps"].tolist() == [2, 8]


def test_cluster_info_rejects_malformed(alvrl, tmp_path):
    p = str(tmp_path / "ci.bin")
    alvrl.write_cluster_info(p, _info())
    raw = open(p, "rb").read()
    for bad in (raw[:-1], raw + b"\0", raw[:20], struct.pack("<Q", 1 << 40) + raw[8:]):
        open(p, "wb").write(bad)
        with pytest.raises(alvrl.AlvrlError):
            alvrl.read_cluster_info(p)
    with pytest.raises(alvrl.AlvrlError):
        alvrl.read_cluster_info(str(tmp_path / "missing.bin"))


def _parse_exr(raw):
    """Independent reading of the single-part scanline layout."""
    assert raw[:4] == bytes([0x76, 0x2F, 0x31, 0x01]) and struct.unpack("<I", raw[4:8])[0] == 2
    o, attrs = 8, {}
    while raw[o] != 0:
        e = raw.index(b"\0", o); name = raw[o:e].decode(); o = e + 1
        e = raw.index(b"\0", o); typ = raw[o:e].decode(); o = e + 1
        n = struct.unpack("<i", raw[o:o + 4])[0]; o += 4
        attrs[name] = (typ, raw[o:o + n]); o += n
    o += 1
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    ch = attrs["channels"][1]
    names, types, q = [], [], 0
    while ch[q] != 0:
        e = ch.index(b"\0", q); names.append(ch[q:e].decode()); q = e + 1
        types.append(struct.unpack("<i", ch[q:q + 4])[0]); q += 16
    offs = struct.unpack(f"<{h}Q", raw[o:o + 8 * h])
    dt = {1: "<f2", 2: "<f4"}[types[0]]
    img = np.zeros((h, w, 3), np.float32)
    for y, off in enumerate(offs):
        yy, size = struct.unpack("<2i", raw[off:off + 8])
        data = np.frombuffer(raw[off + 8:off + 8 + size], dt).reshape(3, w)   # B, G, R
        img[yy] = data[::-1].T
    return attrs, names, types, img


@pytest.mark.parametrize("half", [False, True])
def test_exr_writer(alvrl, tmp_path, half):
    rng = np.random.default_rng(3)
    img = (rng.random((7, 11, 3)) * 4).astype(np.float32)
    img[0, 0] = [0.0, 1e-6, 65000.0]
    p = str(tmp_path / "a.exr")
    alvrl.write_exr(p, img, half=half)
    attrs, names, types, parsed = _parse_exr(open(p, "rb").read())
    assert names == ["B", "G", "R"] and types == [1 if half else 2] * 3
    assert attrs["compression"][1] == b"\0" and attrs["lineOrder"][1] == b"\0"
    want = img.astype(np.float16).astype(np.float32) if half else img
    assert np.array_equal(parsed, want)
    assert np.array_equal(alvrl.read_exr(p), want)


def _rms_reference(a, b, gamma, robust, relative):
    a = np.power(a.astype(np.float64).ravel(), 1.0 / gamma)
    b = np.power(b.astype(np.float64).ravel(), 1.0 / gamma)
    n = a.size
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.where(b == 0, 0.0, (a - b) / b) if relative else a - b
    drop = int(0.5 + n * robust) if robust > 0 else 0
    if drop:
        d = np.sort(d)
    mid = np.sort(d[drop:n - drop] ** 2)
    acc = 0.0
    for x in mid:                     # in order, like the reference's loop
        acc += x
    return np.sqrt(acc / (n - 2 * drop))


@pytest.mark.parametrize("gamma,robust,relative", [(1.0, 0.0, False), (2.2, 0.0, False),
                                                   (1.0, 0.01, False), (1.0, 0.0, True), (2.2, 0.05, True)])
def test_image_rms(alvrl, gamma, robust, relative):
    rng = np.random.default_rng(11)
    ref = rng.random(3000).astype(np.float32)
    ref[::97] = 0
    img = (ref + rng.normal(0, 0.01, ref.size)).clip(0).astype(np.float32)
    got = alvrl.image_rms(img, ref, gamma, robust, relative)
    assert got == pytest.approx(_rms_reference(img, ref, gamma, robust, relative), rel=1e-12, abs=0)
    with pytest.raises(alvrl.AlvrlError):
        alvrl.image_rms(img, ref, 1.0, 0.5)


def test_pass_file_name(alvrl):
    got = alvrl.pass_file_name("/out/smoke", 7, 1.5, 2.25, 0.000125, 123456.0, 4.9e9, 6.0e9)
    want = ("/out/smoke_pass007_precpu1.5000e+00_prewall2.2500e+00_rencpu1.2500e-04_renwall1.2346e+05"
            "_prevrl%.4e_renvrl%.4e.exr" % (np.float32(4.9e9), np.float32(6.0e9)))
    assert got == want


def test_host_header_symbols_exported(alvrl):
    src = open(os.path.join(REPO, "include", "alvrl_host.h")).read()
    names = sorted(set(re.findall(r"ALVRL_API\s+[\w\s\*]+?\b(alvrl_\w+)\s*\(", src)))
    L = alvrl.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert len(names) >= 30 and not missing, missing
