"""HomogeneousMedium's distance-sampling strategies (homogeneous.cpp:150-227):
'balance' (the default), 'single', 'manual' and 'maximum' (MaxExpDist,
maxexp.h:28-94).  The strategy sets the tracer's sampled distances and pdfs
(sampleDistance :275-352, vrlTracer.h:143-213) and the pdfFailure the gather
divides by (eval :354-396, vrlIntegrator.cpp:666-676, 741-751).

CPU part: the oracle's MaxExpDist against the distribution it samples
(closed-form pdf of max_i sigma_i exp(-sigma_i t), integrated numerically),
and the product's host tracer against the oracle, BIT FOR BIT, for every
strategy.  Device gathers and tracer: test_gpu_medium_strategies.py."""
import numpy as np
import pytest

STRATS = [("balance", -1, 0.0), ("single", -1, 0.0), ("single", 0, 0.0), ("manual", -1, 0.7),
          ("maximum", -1, 0.0)]


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def scene_with(alvrl, w, h, strategy, channel, density):
    s = alvrl.scene_default(w, h)
    s.medium.strategy = alvrl.STRATEGIES[strategy]
    s.medium.channel = channel + 1
    s.medium.sampling_density = density
    return s


def test_maxexp_matches_closed_form(oracle):
    """1 - cdf(t) of the oracle's MaxExpDist (pdfFailure with weight 1)
    against the tail of f(t) = max_i s_i exp(-s_i t) / Z by quadrature."""
    m = oracle.medium(weight=1.0, strategy="maximum")
    s = np.array([0.85, 0.65, 0.45], np.float64)
    t = np.linspace(0.0, 40.0, 400001)
    f = (s[:, None] * np.exp(-s[:, None] * t[None])).max(0)
    z = np.trapezoid(f, t)
    tail = z - np.concatenate([[0.0], np.cumsum((f[1:] + f[:-1]) * 0.5 * np.diff(t))])
    for d in (0.0, 0.1, 0.5, 1.3, 2.0, 4.0, 9.0):
        _, pf = oracle.medium_eval(m, d)
        k = int(round(d / 1e-4))
        assert abs(pf - tail[k] / z) < 2e-5, (d, pf, tail[k] / z)
    # the balance pdf for comparison is a different function
    _, pfb = oracle.medium_eval(oracle.medium(weight=1.0), 1.3)
    assert abs(pfb - oracle.medium_eval(m, 1.3)[1]) > 1e-3


def test_single_and_manual_eval(oracle):
    """pdfFailure of 'single' (the smallest sigma_t by default, or the given
    channel) and 'manual' is exp(-density d), mixed with the sampling weight."""
    for strategy, channel, density, expect in (("single", -1, 0.0, 0.45), ("single", 0, 0.0, 0.85),
                                               ("manual", -1, 0.7, 0.7)):
        m = oracle.medium(strategy=strategy, channel=channel, density=density)
        assert m.density == pytest.approx(expect)
        tr, pf = oracle.medium_eval(m, 1.7)
        w = m.sampling_weight
        assert pf == pytest.approx(w * np.exp(-expect * 1.7) + (1 - w), rel=1e-6)
        assert tr == pytest.approx(list(np.exp(-np.array([0.85, 0.65, 0.45]) * 1.7)), rel=1e-6)


def test_maximum_needs_distinct_sigma_t(oracle, alvrl):
    with pytest.raises(ValueError):
        oracle.medium(sigma_s=(0.6, 0.6, 0.4), strategy="maximum")
    s = alvrl.scene_default(8, 8)
    s.medium.sigma_s[0] = s.medium.sigma_s[1]
    s.medium.strategy = alvrl.STRATEGIES["maximum"]
    with pytest.raises(alvrl.AlvrlError):
        alvrl.trace_vrls(s, 10)


@pytest.mark.parametrize("strategy,channel,density", STRATS)
@pytest.mark.parametrize("short", [True, False])
def test_tracer_strategies_match_oracle(alvrl, oracle, strategy, channel, density, short):
    """The host tracer under every strategy == the oracle's, bit for bit, and
    the strategies give different VRL sets (they are not ignored)."""
    s = scene_with(alvrl, 16, 16, strategy, channel, density)
    m = oracle.medium(strategy=strategy, channel=channel, density=density)
    mine, pc = alvrl.trace_vrls(s, 2000, seed=0x5EED0001, short_vrls=short)
    ref, rpc = oracle.trace(oracle.scene(16, 16), m, 2000, seed=0x5EED0001, short_vrls=short)
    assert pc == rpc
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    if strategy != "balance":
        base, _ = alvrl.trace_vrls(alvrl.scene_default(16, 16), 2000, seed=0x5EED0001, short_vrls=short)
        assert base.shape != mine.shape or not np.array_equal(base, mine)


def test_strategies_unbiased_vrl_power(oracle):
    """Every strategy estimates the same light transport: the mean total VRL
    power per particle (scattered power in the medium, a tracer expectation)
    agrees across strategies within sampling error."""
    sc = oracle.scene(8, 8)
    means = {}
    for strategy, channel, density in STRATS:
        m = oracle.medium(strategy=strategy, channel=channel, density=density)
        v, pc = oracle.trace(sc, m, 60000, seed=0x1234, short_vrls=True)
        means[strategy + str(channel)] = v[6:9].sum() / pc
    vals = np.array(list(means.values()))
    assert np.all(np.abs(vals / vals.mean() - 1) < 0.05), means
