"""Checkpoint / resume of the vectorised trainer: a trainer restored from
VecTrainer.state_dict() — through torch.save / torch.load(weights_only=True) — continues bit for
bit as the uninterrupted one: per-env SoA state, replay ring, every network and Adam moment."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _snapshot(tr):
    e = tr.env
    snap = {k: getattr(e, k).clone() for k in tr.ENV_STATE}
    snap["replay"] = tr.replay.rows.clone()
    for name, net in tr.td3.networks().items():
        snap[name] = net.params.clone()
        snap[name + "_packed"] = net.packed.clone()
    for name, o in (("adam_a", tr.td3.actor_optimizer), ("adam_c1", tr.td3.critic_optimizer_1),
                    ("adam_c2", tr.td3.critic_optimizer_2)):
        snap[name + "_m"], snap[name + "_v"] = o.m.clone(), o.v.clone()
    snap["action"] = tr.action.clone()
    return snap


@pytest.mark.parametrize("demos", [True, False])
def test_resume_is_bit_identical(tmp_path, demos):
    from nav import _lib
    from nav.trainer import VecTrainer
    _lib.require_gpu()
    torch.cuda.set_device(0)
    kw = dict(n_envs=4096, hidden=64, n_hidden=2, batch=2048, updates_per_step=2,
              envs_per_group=1024, demos=demos, device=DEV)
    a = VecTrainer(**kw)
    for _ in range(5):  # learner active from the first step with a full batch in the ring
        a.step()
    path = os.path.join(tmp_path, "trainer.pt")
    a.save(path)
    for _ in range(4):
        a.step()
    torch.cuda.synchronize()
    want = _snapshot(a)

    b = VecTrainer.load(path, device=DEV)
    assert b.steps == 5 and b.replay.position == (5 * 4096) % b.replay.capacity
    for _ in range(4):
        b.step()
    torch.cuda.synchronize()
    got = _snapshot(b)
    assert b.steps == a.steps and b.td3.update_counter == a.td3.update_counter
    assert (b.replay.position, b.replay.size) == (a.replay.position, a.replay.size)
    for k, v in want.items():
        assert torch.equal(got[k], v), k
    # the resumed run really moved: the learner and the envs changed after the checkpoint
    sd = torch.load(path, weights_only=True)
    assert not torch.equal(sd["env"]["state"], want["state"].cpu())
    assert not torch.equal(sd["td3"]["critic1"]["params"], want["critic1"].cpu())
