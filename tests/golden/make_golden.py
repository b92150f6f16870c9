"""Generate the committed golden fixtures of the ALVRL hot path.

The reference (Mitsuba 0.6 + Boost + Xerces) cannot be built in this image and
ships no golden vectors for this path, so these
fixtures come from the CPU restatement in oracle/ (which follows the
reference's files line by line, cited there).  They pin the restatement and
the device path against a fixed record of its outputs; they do NOT pin the
restatement against the reference itself ("parity unpinned" beyond the
Philox4x32-10 known answers of Random123, tests/test_oracle.py).

    python tests/golden/make_golden.py      # rewrites the files next to it

Files:
  vrls_c1.txt     256 VRLs of the smoke box, reference ASCII format
                  (VRL.h:43-54: "sx sy sz ex ey ez r g b" per line)
  kats.npz        per-function known answers: getClosestPoints,
                  KullaSampling, sampleVtoDistance, HomogeneousMedium::eval
  c1_small.npz    48x32 smoke box with vrls_c1.txt (particleCount = #lines,
                  VRL.h:127): brute-force frame, R rows of 16 pixels, and the
                  LightSlice outputs (slice map, representatives, per-slice
                  clusters) and the clustered frame at 12 slices
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4
W, H = 48, 32
NVRL = 256
NSLICES = 12


def read_vrl_ascii(path):
    rows = [list(map(float, l.split())) for l in open(path) if l.strip()]
    return np.ascontiguousarray(np.array(rows, np.float32).T)


def kats(o):
    rng = np.random.default_rng(20261015)
    out = {}
    # getClosestPoints: random segment pairs + parallel / clamped / crossing cases
    cp_in = rng.uniform(-1, 1, size=(64, 4, 3)).astype(np.float32)
    cp_in[0] = [[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]]           # parallel
    cp_in[1] = [[0, 0, 0], [1, 0, 0], [0.5, -1, 0], [0.5, 1, 0]]      # crossing
    cp_in[2] = [[0, 0, 0], [1, 0, 0], [2, 1, 0], [3, 2, 0]]           # clamped at ends
    cp_in[3] = [[0, 0, 0], [1, 0, 0], [-1, 1, 1], [-1, 1, 1]]         # degenerate 2nd segment
    cp_out = np.zeros((64, 7), np.float32)
    for i, c in enumerate(cp_in):
        h, a, b = o.closest_points(*c)
        cp_out[i] = [h] + a + b
    out["closest_in"], out["closest_out"] = cp_in, cp_out
    # KullaSampling: A, B, D, u
    ku_in = rng.uniform(-1, 1, size=(64, 10)).astype(np.float32)
    ku_in[:, 9] = rng.uniform(0, 1, 64)
    ku_in[0] = [0, 0, 0, 0, 0, 2, 1, 0, 1, 0.5]                        # symmetric: pdf 2/pi
    ku_in[1] = [0, 0, 0, 0, 0, 1, 0.1, 0, 3, 0.25]                     # D beyond B
    ku_in[2] = [0, 0, 0, 0, 0, 1, 1e-3, 0, 0.5, 0.999]                 # D near the line
    ku_out = np.zeros((64, 4), np.float32)
    for i, k in enumerate(ku_in):
        pdf, r = o.kulla(k[0:3], k[3:6], k[6:9], float(k[9]))
        ku_out[i] = [pdf] + r
    out["kulla_in"], out["kulla_out"] = ku_in, ku_out
    # sampleVtoDistance: E, d (unit), hit p, S, End, u
    sv_in = np.zeros((64, 16), np.float32)
    for i in range(64):
        E = rng.uniform(-0.9, 0.9, 3)
        d = rng.normal(size=3); d /= np.linalg.norm(d)
        p = E + d * rng.uniform(0.5, 2.0)
        S = rng.uniform(-0.9, 0.9, 3); End = S + rng.normal(size=3) * 0.5
        sv_in[i] = np.concatenate([E, d, p, S, End, [rng.uniform()]])
    sv_in[0, 9:12] = sv_in[0, 12:15]                                    # zero-length VRL
    sv_in[1, 3:6] = (0, 0, 1); sv_in[1, 12:15] = sv_in[1, 9:12] + (0, 0, 0.7)   # parallel
    sv_out = np.zeros((64, 4), np.float32)
    for i, s in enumerate(sv_in):
        pdf, V = o.sample_v_to_distance(s[0:3], s[3:6], s[6:9], s[9:12], s[12:15], float(s[15]))
        sv_out[i] = [pdf] + V
    out["svd_in"], out["svd_out"] = sv_in, sv_out
    # HomogeneousMedium::eval (balance strategy), default and HG media
    dists = np.array([0, 1e-6, 0.01, 0.5, 1, 2, 10, 60, 100, 1e3], np.float32)
    me = np.zeros((2, len(dists), 4), np.float32)
    for j, m in enumerate([o.medium(), o.medium(sigma_s=(1.5, 0.2, 0.0), sigma_a=(0.1, 0.0, 0.3))]):
        for i, dd in enumerate(dists):
            tr, pf = o.medium_eval(m, float(dd))
            me[j, i] = tr + [pf]
    out["medium_dist"], out["medium_out"] = dists, me
    return out


def c1_small(o, vrls):
    from oracle import Prep
    pc = vrls.shape[1]                       # particleCount = size() for file VRLs
    sc = o.scene(W, H)
    m = o.medium()
    recs = o.records(sc)
    P = o.params(m, seed=SEED_RNG)
    brute, _ = o.gather_brute(P, recs, vrls, pc)
    rows = np.arange(0, W * H, (W * H) // 16, dtype=np.uint32)[:16]
    _, Rrows, _ = o.gather_brute(P, recs[rows], vrls, pc, rec_ids=rows, domain=2, want_R=True)
    # LightSlice at NSLICES slices (adaptive local refinement, ALVRL defaults otherwise)
    prep = Prep(o, o.prep_params(seed=SEED_RNG, pass_=0, target_num_slices=NSLICES))
    p2s = prep.build_slices(sc)
    off, pix, su, gu = prep.sample_slice_mapping(64.0, W * H)
    xs, ys = pix // H, pix % H                                   # column-major ids
    rep_ids = (ys * W + xs).astype(np.uint32)
    _, R, _ = o.gather_brute(P, recs[rep_ids], vrls, pc, rec_ids=rep_ids, domain=2, want_R=True)
    cl = prep.build_clusters(np.ascontiguousarray(R.transpose(1, 0, 2)))
    pid = np.arange(W * H, dtype=np.uint32)
    sl = p2s[(pid % W) * H + pid // W]
    clustered, _ = o.gather_clustered(P, recs, sl, vrls, pc, cl["slice_off"], cl["reps"],
                                      cl["weights"], cl["fb_reps"], cl["fb_weights"], rec_ids=pid)
    return dict(brute=brute, R_rows=rows, R=Rrows, slices=p2s, rep_off=off, rep_pix=pix,
                slice_under=su, global_under=np.float32(gu), cl_slice_off=cl["slice_off"],
                cl_reps=cl["reps"], cl_weights=cl["weights"], cl_fb_reps=cl["fb_reps"],
                cl_fb_weights=cl["fb_weights"], clustered=clustered)


def main():
    from oracle import Oracle
    o = Oracle()
    sc = o.scene(W, H)
    vrls, _ = o.trace(sc, o.medium(), NVRL, seed=SEED_VRL)
    vrls = vrls[:, :NVRL]
    path = os.path.join(HERE, "vrls_c1.txt")
    with open(path, "w") as f:
        for i in range(vrls.shape[1]):
            f.write(" ".join("%.9g" % float(x) for x in vrls[:, i]) + "\n")
    vrls = read_vrl_ascii(path)                  # exactly what a reader of the file sees
    np.savez_compressed(os.path.join(HERE, "kats.npz"), **kats(o))
    np.savez_compressed(os.path.join(HERE, "c1_small.npz"), **c1_small(o, vrls))
    print("wrote vrls_c1.txt, kats.npz, c1_small.npz")


if __name__ == "__main__":
    main()
