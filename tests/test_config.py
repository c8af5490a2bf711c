"""Config layer: this repo's cfgs and the reference's unmodified cfg resolve with the reference's
resolvers and types (script/run.py:18-20)."""
import os

import pytest

from diffusionpolicyoptimization_amd.util.config import apply_overrides, get_class, load_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CFG = "/root/reference/cfg/gym/finetune/hopper-v2"


@pytest.mark.parametrize("sub,name,do,envs", [("hopper-v2", "ft_ppo_diffusion_mlp", 11, 4),
                                               ("hopper-v2", "ft_ppo_diffusion_mlp_64env", 11, 64),
                                               ("walker2d-v2", "ft_ppo_diffusion_mlp", 17, 256),
                                               ("halfcheetah-v2", "ft_ppo_diffusion_mlp", 17, 2048)])
def test_repo_cfgs(sub, name, do, envs):
    c = load_config(os.path.join(ROOT, "cfg/gym/finetune", sub), name)
    assert c.model.actor.cond_dim == do and isinstance(c.model.actor.cond_dim, int)
    assert c.env.n_envs == envs and c.model.critic.cond_dim == do
    assert get_class(c._target_).__name__ == "TrainPPODiffusionAgent"
    assert get_class(c.model._target_).__name__ == "PPODiffusion"
    assert c.train.actor_lr == 1e-4 and c.env.wrappers.multi_step.n_action_steps == 4


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference not mounted (build container only)")
def test_reference_cfg_is_drop_in(monkeypatch):
    monkeypatch.setenv("DPPO_LOG_DIR", "/tmp/log")
    monkeypatch.setenv("DPPO_DATA_DIR", "/tmp/data")
    c = load_config(REF_CFG, "ft_ppo_diffusion_mlp", ["train.n_steps=7"])
    assert c.train.n_steps == 7 and c.model.actor.cond_dim == 11
    assert c.logdir.startswith("/tmp/log/gym-finetune/hopper-medium-v2_ppo_diffusion_mlp_ta4_td20_tdf10/")
    for t in (c._target_, c.model._target_, c.model.actor._target_, c.model.critic._target_):
        assert get_class(t).__module__.startswith("diffusionpolicyoptimization_amd.")


def test_overrides_and_resolvers():
    c = apply_overrides({"a": {"b": 1}}, ["a.b=2", "+a.c=[1,2]", "x=hello"])
    assert c.a.b == 2 and c.a.c == [1, 2] and c.x == "hello"
    from diffusionpolicyoptimization_amd.util.config import resolve
    r = resolve({"n": 3, "k": "${eval:'${n} * 2'}", "s": "v${n}_${k}", "u": "${round_up:2.2}"})
    assert r.k == 6 and r.s == "v3_6" and r.u == 3
