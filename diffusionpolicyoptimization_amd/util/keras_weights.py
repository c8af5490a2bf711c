"""Keras-3 `save_weights` layouts of the reference's models, over util/h5.py.

Keras 3 writes a model's variables as datasets `<attribute path>/vars/<i>` (a Dense layer: vars/0
= kernel [in, out], vars/1 = bias): child objects are walked in sorted attribute order, a layer
held in a list/Sequential is named by its snake-cased class name with a per-container count
(dense, dense_1, ...), and an object already written (the reference's `network` IS `actor`) is not
written twice. For the reference's classes that gives:
  DiffusionMLP (model/diffusion/mlp_diffusion.py:40-62): time_embedding/layers/{dense,dense_1},
      mlp_mean/{input_layer, residual_blocks/two_layer_pre_activation_res_net_linear/{l1,l2},
      output_layer}   — the root of a pretrain checkpoint (agent/pretrain/train_agent.py:150-154)
      and of network_path (diffusion_vpg.py:85-97);
  CriticObs (model/common/critic.py:33): Q1/... (same ResidualMLP names);
  PPODiffusion (agent/finetune/train_agent.py:127-133): actor/, actor_ft/, critic/.
Reading is tolerant of the container names (any residual block / the Sequential's Dense layers in
Keras's numbering) and checks every shape against the flat spec; what is missing is named in the
error. Parity is pinned to this published layout, not to a file Keras wrote (TF/Keras cannot be
installed here): the reader itself is pinned to files a real HDF5 library wrote.
"""
import logging
import re

import numpy as np

from .h5 import read_h5, write_h5

BLOCK = "two_layer_pre_activation_res_net_linear"


def _dense_paths(prefix):
    """Keras-3 paths of a ResidualMLP with one residual block under `prefix`."""
    return {"in": f"{prefix}input_layer", "l1": f"{prefix}residual_blocks/{BLOCK}/l1",
            "l2": f"{prefix}residual_blocks/{BLOCK}/l2", "out": f"{prefix}output_layer"}


def actor_paths(prefix=""):
    """flat-spec name -> dataset path (ops.actor_param_spec names)."""
    p = _dense_paths(prefix + "mlp_mean/")
    te = prefix + "time_embedding/layers/"
    out = {"time_w1": te + "dense/vars/0", "time_b1": te + "dense/vars/1",
           "time_w2": te + "dense_1/vars/0", "time_b2": te + "dense_1/vars/1"}
    for k, v in p.items():
        out[f"{k}_w"], out[f"{k}_b"] = v + "/vars/0", v + "/vars/1"
    return out


def critic_paths(prefix=""):
    out = {}
    for k, v in _dense_paths(prefix + "Q1/").items():
        out[f"{k}_w"], out[f"{k}_b"] = v + "/vars/0", v + "/vars/1"
    return out


def _keras_index(name):
    m = re.fullmatch(r"(.*?)(?:_(\d+))?", name)
    return (m.group(1), int(m.group(2) or 0))


def _resolve(data, want, used=None):
    """want: name -> canonical path. Container-named levels (the residual block, the Sequential's
    Dense layers) are matched by structure when the canonical name is absent. `used` collects the
    dataset paths read."""
    got, missing = {}, []
    used = set() if used is None else used
    for name, path in want.items():
        if path in data:
            got[name] = data[path]
            used.add(path)
            continue
        alt = None
        if "/residual_blocks/" in path:                      # any single residual block name
            head, tail = path.split("/residual_blocks/", 1)
            tail = tail.split("/", 1)[1]
            cands = sorted({k.split("/residual_blocks/", 1)[1].split("/", 1)[0] for k in data
                            if k.startswith(head + "/residual_blocks/")})
            if len(cands) == 1:
                alt = f"{head}/residual_blocks/{cands[0]}/{tail}"
        elif "/time_embedding/layers/" in path or path.startswith("time_embedding/layers/"):
            head, tail = path.rsplit("/layers/", 1)
            which = 0 if tail.startswith("dense/") else 1
            layers = sorted({k[len(head) + 8:].split("/", 1)[0] for k in data
                             if k.startswith(head + "/layers/") and k.endswith("/vars/0") and data[k].ndim == 2},
                            key=_keras_index)
            if len(layers) == 2:
                alt = f"{head}/layers/{layers[which]}/{tail.split('/', 1)[1]}"
        if alt is not None and alt in data:
            got[name] = data[alt]
            used.add(alt)
        else:
            missing.append(path)
    return got, missing


def _datasets(data, prefixes):
    return sorted(k for k in data if k != "__groups__" and any(k.startswith(p) for p in prefixes))


def _check_unused(path, data, used, model_prefixes, what):
    """Every dataset inside the model's own subtrees must have been read: a Keras file whose layout
    differs from the one this reader follows (renamed or extra variables) fails here, naming them,
    instead of loading with variables silently skipped. Datasets outside those subtrees (e.g.
    optimizer state) are listed in the log."""
    unread = [k for k in _datasets(data, model_prefixes) if k not in used]
    if unread:
        raise ValueError(f"{path}: {what}: datasets inside the model that this reader does not map (layout "
                         f"differs from the Keras-3 layout in util/keras_weights.py): {unread[:50]}")
    other = [k for k in data if k != "__groups__" and k not in used and not any(k.startswith(p) for p in model_prefixes)]
    if other:
        logging.getLogger(__name__).warning("%s: ignoring %d dataset(s) outside the %s: %s", path, len(other), what,
                                            other[:20])


def _find_prefix(data, candidates, probe):
    for p in candidates:
        if any(k.startswith(p + probe) for k in data):
            return p
    return None


def _checked(got, spec, what, path):
    out = {}
    for name, shape in spec:
        a = np.asarray(got[name], np.float32)
        if a.shape != tuple(shape):
            raise ValueError(f"{path}: {what} variable {name} has shape {a.shape}, the model needs {tuple(shape)}")
        out[name] = a
    return out


def load_actor(path, spec, prefixes=("", "network/", "actor/", "actor_ft/")):
    """A DiffusionMLP's weights from a Keras-3 weights file -> {flat-spec name: array}. The file
    may hold the network at its root (a pretrain checkpoint / network_path) or inside a model
    (first match of `prefixes`)."""
    data = read_h5(path)
    p = _find_prefix(data, prefixes, "mlp_mean/")
    if p is None:
        raise ValueError(f"{path}: no DiffusionMLP (mlp_mean/...) found; datasets: "
                         + ", ".join(sorted(k for k in data if k != "__groups__"))[:2000])
    used = set()
    got, missing = _resolve(data, actor_paths(p), used)
    if missing:
        raise ValueError(f"{path}: missing DiffusionMLP variables: {missing}")
    _check_unused(path, data, used, (p + "mlp_mean/", p + "time_embedding/"), "DiffusionMLP")
    return _checked(got, spec, "actor", path)


ETA_LOGIT = "eta/vars/0"                 # EtaFixed's one variable, where Keras 3 writes a sub-layer's weight
ETA_OPT = "eta/optimizer_state"         # [m, v, step] of its AdamW (resume exactly)


def load_ppo_model(path, actor_spec, critic_spec):
    """{"actor", "actor_ft", "critic"} dicts from a fine-tune checkpoint (PPODiffusion.save_weights),
    plus "eta" = {"logit", "m", "v", "step"} when the model learned eta."""
    data = read_h5(path)
    out = {}
    used = set()
    if ETA_LOGIT in data:
        opt = np.asarray(data.get(ETA_OPT, np.zeros(3)), np.float64).reshape(-1)
        out["eta"] = {"logit": float(np.asarray(data[ETA_LOGIT]).reshape(-1)[0]), "m": float(opt[0]),
                      "v": float(opt[1]), "step": int(opt[2])}
        used.update(k for k in (ETA_LOGIT, ETA_OPT) if k in data)
    for key, paths, spec in (("actor", actor_paths("actor/"), actor_spec),
                             ("actor_ft", actor_paths("actor_ft/"), actor_spec),
                             ("critic", critic_paths("critic/"), critic_spec)):
        got, missing = _resolve(data, paths, used)
        if missing:
            raise ValueError(f"{path}: missing {key} variables: {missing}")
        out[key] = _checked(got, spec, key, path)
    _check_unused(path, data, used, ("actor/", "actor_ft/", "critic/"), "PPODiffusion model")
    return out


def _empty_groups(prefix, network):
    """The (empty) `vars` groups Keras writes for every saveable without variables of its own."""
    g = [prefix + "vars"]
    if network == "actor":
        g += [prefix + "mlp_mean/vars", prefix + f"mlp_mean/residual_blocks/{BLOCK}/vars",
              prefix + "time_embedding/vars", prefix + "time_embedding/layers/sinusoidal_pos_emb/vars"]
    else:
        g += [prefix + "Q1/vars", prefix + f"Q1/residual_blocks/{BLOCK}/vars"]
    return g


def save_actor(path, params):
    """A DiffusionMLP at the file root (agent/pretrain/train_agent.py:150-154 layout)."""
    write_h5(path, {actor_paths("")[k]: np.asarray(v, np.float32) for k, v in params.items()},
             groups=_empty_groups("", "actor"))


def save_ppo_model(path, actor, actor_ft, critic, eta=None):
    """PPODiffusion.save_weights (agent/finetune/train_agent.py:127-133 layout); eta: the learnable
    eta's {"logit", "m", "v", "step"} (learn_eta models), stored under eta/."""
    d = {}
    if eta is not None:
        d[ETA_LOGIT] = np.array([eta["logit"]], np.float32)
        d[ETA_OPT] = np.array([eta["m"], eta["v"], eta["step"]], np.float64)
    for prefix, params, paths in (("actor/", actor, actor_paths("actor/")),
                                  ("actor_ft/", actor_ft, actor_paths("actor_ft/")),
                                  ("critic/", critic, critic_paths("critic/"))):
        for k, v in params.items():
            d[paths[k]] = np.asarray(v, np.float32)
    groups = ["vars"] + _empty_groups("actor/", "actor") + _empty_groups("actor_ft/", "actor") + \
        _empty_groups("critic/", "critic") + (["eta"] if eta is not None else [])
    write_h5(path, d, groups=groups)
