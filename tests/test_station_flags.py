"""mceik_mcmc_init's station contract (host-side checks, no GPU): Cartesian
coordinates only (mceik_stations_struct.lcartesian = 1, as homog.c:121 sets
it), and a used pick needs its station's phase flag (lhasP / lhasS,
mceik_struct.h:43-46; homog.c:313-335 builds tables only for flagged
stations).  Both refusals happen before the library touches a device."""
import numpy as np
import pytest

from mceik_amd import mcmc


def _problem(phases="P"):
    return mcmc.make_problem("C2", n=16, nstat=4, nev=3, phases=phases, picks="analytic")


def test_flags_follow_used_picks():
    p = _problem("PS")
    hp, hs = p.station_flags()
    assert hp.all() and hs.all() and p.skip.shape == (2, 4) and not p.skip.any()
    p.luse[(p.pick_type == mcmc.S_PRIMARY_PICK) & (p.obs_stat == 2)] = 0
    hp, hs = p.station_flags()
    assert list(hs) == [1, 1, 0, 1] and p.skip[1, 2] == 1 and p.skip.sum() == 1


def test_geographic_stations_refused(capfd):
    p = _problem()
    p.lcartesian = 0
    with pytest.raises(RuntimeError, match=r"failed \(1\)"):
        mcmc.Sampler(p, nchains=1)
    assert "lcartesian = 0" in capfd.readouterr().err


@pytest.mark.parametrize("flag", ["has_p", "has_s"])
def test_used_pick_without_station_flag_refused(flag, capfd):
    p = _problem("PS")
    setattr(p, flag, np.array([1, 0, 1, 1], np.int32))     # station 2 (1-based) has picks of that phase
    with pytest.raises(RuntimeError, match=r"failed \(1\)"):
        mcmc.Sampler(p, nchains=1)
    err = capfd.readouterr().err
    assert "station 2 (1-based)" in err and ("lhasP" if flag == "has_p" else "lhasS") in err
