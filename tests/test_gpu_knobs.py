"""GPU parity of the reference's config knobs through every launch shape (C ABI, libmev.so):
movement_params.reset_rng_episode = False (movement.py:16-18), EP_MAX_TIME != ep_time
(base.py:105-109,126,407-409) and non-default utility_params (utilities.py:44-55), against
fixtures the reference wrote (tests/golden/knob_*.npz; tests/test_knobs.py pins the oracle to
the same files and checks the lowering).

Launch shapes per fixture:
  single  -- one launch per step (mev_step(1); k_step_packed / k_steps_block), float64 outputs
  fused   -- mev_step(7): seven steps per launch, the state in registers between them
  rollout -- mev_rollout over every step, float64 outputs (k_steps_packed / k_steps_block)
  scale   -- lean rollout over a replicated batch (env i runs seed i % n) big enough for the
             large-batch kernels: the two-group k_steps_lds2 (U = 15 / 30 with the episode draw
             table), the persistent LDS-table k_steps_packed (no table: reset_rng_episode off)
Bars: positions, serving indices, done flags and float64 rates bit-exact; float64 utilities
to 1e-12; float32 obs rate / utility and the reward to 1e-5 relative (north_star)."""
import numpy as np
import pytest

from helpers import KNOB_FIXTURES, knob_done, knob_engine, load, synced_pcg

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _check_host(d, name, s, idx, obs, srv, rew, done, rate64=None, util64=None, met=None,
                xy=None):
    tag = f"{name} step {s}"
    W = 200.0
    if xy is None:
        xy = np.rint(obs[..., :2] * W).astype(np.int64)
    np.testing.assert_array_equal(xy, d["xy"][idx, s], err_msg=tag + " positions")
    np.testing.assert_array_equal(srv, d["serving"][idx, s], err_msg=tag + " serving")
    np.testing.assert_allclose(obs[..., 2], d["rate"][idx, s].astype(np.float32), rtol=RTOL,
                               err_msg=tag + " rate")
    ru = d["util"][idx, s]
    act = ~np.isnan(ru)
    np.testing.assert_allclose(obs[..., 3][act], ru[act].astype(np.float32), rtol=RTOL, atol=0,
                               err_msg=tag + " utility")
    np.testing.assert_allclose(rew, d["metrics"][idx, s, 2], rtol=RTOL, atol=0,
                               err_msg=tag + " reward")
    np.testing.assert_array_equal(done.astype(bool), np.full(len(done), knob_done(d)[s]),
                                  err_msg=tag + " done")
    if rate64 is not None:
        np.testing.assert_array_equal(rate64, d["rate"][idx, s], err_msg=tag + " rate64")
        np.testing.assert_allclose(util64[act], ru[act], rtol=1e-12, atol=1e-15,
                                   err_msg=tag + " util64")
        np.testing.assert_array_equal(met[:, :2], d["metrics"][idx, s, :2], err_msg=tag + " met")
        np.testing.assert_allclose(met[:, 3], d["metrics"][idx, s, 3], rtol=RTOL)


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_knob_single_launches(name):
    d = load(name)
    n = len(d["seeds"])
    idx = np.arange(n)
    eng = knob_engine(d, rate64=True, util64=True, metrics=True, fuse_steps=-1)
    for s in range(d["xy"].shape[1]):
        eng.step()
        _check_host(d, name, s, idx, eng.obs.cpu().numpy(), eng.serving.cpu().numpy(),
                    eng.reward.cpu().numpy(), eng.done.cpu().numpy(), eng.rate64.cpu().numpy(),
                    eng.util64.cpu().numpy(), eng.metrics.cpu().numpy(),
                    xy=eng.ue_xy.cpu().numpy())
    eng.close()


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_knob_fused_steps(name):
    """mev_step(7) launches (chunks cross the episode ends): the outputs of each launch's last
    step and the state after it."""
    d = load(name)
    n = len(d["seeds"])
    idx = np.arange(n)
    S = d["xy"].shape[1]
    eng = knob_engine(d, rate64=True, util64=True, metrics=True)
    s = 0
    while s < S:
        k = min(7, S - s)
        eng.step(k)
        s += k
        _check_host(d, name, s - 1, idx, eng.obs.cpu().numpy(), eng.serving.cpu().numpy(),
                    eng.reward.cpu().numpy(), eng.done.cpu().numpy(), eng.rate64.cpu().numpy(),
                    eng.util64.cpu().numpy(), eng.metrics.cpu().numpy(),
                    xy=eng.ue_xy.cpu().numpy())
    eng.close()


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_knob_rollout_exact(name):
    d = load(name)
    n = len(d["seeds"])
    idx = np.arange(n)
    S = d["xy"].shape[1]
    eng = knob_engine(d, rate64=True, util64=True, metrics=True)
    tr = eng.rollout(S)
    for s in range(S):
        _check_host(d, name, s, idx, tr.obs[s].cpu().numpy(), tr.serving[s].cpu().numpy(),
                    tr.reward[s].cpu().numpy(), tr.done[s].cpu().numpy(),
                    tr.rate64[s].cpu().numpy(), tr.util64[s].cpu().numpy(),
                    tr.metrics[s].cpu().numpy())
    np.testing.assert_array_equal(eng.ue_xy.cpu().numpy(), d["xy"][:, S - 1])
    eng.close()


def _scale_envs(U):
    # enough env pairs for k_steps_lds2 (4,096 pairs per 256 resident workgroups; a partial last
    # pair), else a batch that spreads over every CU
    return {30: 16390, 15: 32774}.get(U, 2053 if U <= 64 else 96)


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_knob_lean_rollout_at_scale(name):
    """The bench's launch shape (lean outputs, trajectory rows) over a replicated batch: every
    replica equals its seed's reference run, compared on the device row by row; the final
    state equals the one-step launches' (synced stream states included)."""
    import torch
    d = load(name)
    n = len(d["seeds"])
    U = d["xy"].shape[2]
    S = d["xy"].shape[1]
    E = _scale_envs(U)
    eng = knob_engine(d, num_envs=E)
    tr = eng.rollout(S)
    dev = eng.device
    idx = torch.arange(E, device=dev) % n
    done = knob_done(d)
    for s in range(S):
        srv = torch.from_numpy(d["serving"][:, s]).to(dev)[idx]
        assert torch.equal(tr.serving[s].long(), srv), f"{name} step {s} serving"
        xy = torch.from_numpy(d["xy"][:, s]).to(dev)[idx]
        assert torch.equal(torch.round(tr.obs[s, ..., :2] * 200.0).long(), xy), f"{name} {s} xy"
        rate = torch.from_numpy(d["rate"][:, s]).to(dev)[idx].float()
        torch.testing.assert_close(tr.obs[s, ..., 2], rate, rtol=RTOL, atol=0)
        ru = torch.from_numpy(d["util"][:, s]).to(dev)[idx].float()
        act = ~torch.isnan(ru)
        torch.testing.assert_close(tr.obs[s, ..., 3][act], ru[act], rtol=RTOL, atol=0)
        rew = torch.from_numpy(d["metrics"][:, s, 2]).to(dev)[idx].float()
        torch.testing.assert_close(tr.reward[s], rew, rtol=RTOL, atol=0)
        assert bool((tr.done[s] == int(done[s])).all()), f"{name} step {s} done"
    final = [eng.ue_state.clone(), synced_pcg(eng).clone(), eng.t.clone()]
    eng.close()
    # the same replicated batch through one-step launches: the same final state
    ref = knob_engine(d, num_envs=E, fuse_steps=-1)
    for _ in range(S):
        ref.step()
    for a, b in zip(final, [ref.ue_state, synced_pcg(ref), ref.t]):
        assert torch.equal(a, b)
    ref.close()
