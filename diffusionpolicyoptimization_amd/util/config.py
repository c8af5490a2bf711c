"""Minimal Hydra/OmegaConf-compatible config layer (Hydra 1.3 and OmegaConf 2.3 are not installed
on MI355X hosts here; reference script/run.py:18-41 and cfg/ rely on them).

Supported: YAML loading (safe loader), `defaults: [_self_]`, the `hydra:` block (ignored),
interpolations ${a.b}, ${eval:'...'}, ${round_up:x}, ${round_down:x} (script/run.py:18-20),
${oc.env:VAR[,default]}, ${now:fmt}; Hydra-style CLI overrides key=value / +key=value / ~key;
recursive `_target_` instantiation where the reference's dotted class paths
(agent.finetune..., model.diffusion..., model.common...) map onto this package.
"""
import ast
import datetime
import importlib
import math
import os
import re

import yaml

PACKAGE = "diffusionpolicyoptimization_amd"


class _Loader(yaml.SafeLoader):
    """SafeLoader + YAML 1.2 floats (1e-4 without a dot), as OmegaConf's loader reads them."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                |\.[0-9_]+(?:[eE][-+][0-9]+)?
                |[-+]?\.(?:inf|Inf|INF)
                |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))
_NOW = datetime.datetime.now()


class Cfg(dict):
    """dict with attribute access (the subset of DictConfig the agent uses)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def get(self, k, default=None):
        v = dict.get(self, k, default)
        return default if v is None and default is not None else v


def to_cfg(x):
    if isinstance(x, dict):
        return Cfg({k: to_cfg(v) for k, v in x.items()})
    if isinstance(x, list):
        return [to_cfg(v) for v in x]
    return x


def to_container(x):
    if isinstance(x, dict):
        return {k: to_container(v) for k, v in x.items()}
    if isinstance(x, list):
        return [to_container(v) for v in x]
    return x


_INTERP = re.compile(r"\$\{([^${}]*)\}")


def _lookup(root, path):
    node = root
    for part in path.split("."):
        if isinstance(node, list):
            node = node[int(part)]
        else:
            node = node[part]
    return node


def _resolver(expr, root):
    if ":" in expr and not expr.startswith("."):
        name, arg = expr.split(":", 1)
        if name == "eval":
            arg = arg.strip()
            if arg[:1] in "'\"" and arg[-1:] == arg[:1]:
                arg = arg[1:-1]
            return eval(arg, {"math": math}, {})  # cfg-author expressions, as in script/run.py:18
        if name == "round_up":
            return math.ceil(float(arg))
        if name == "round_down":
            return math.floor(float(arg))
        if name == "oc.env":
            var, _, default = arg.partition(",")
            v = os.environ.get(var.strip())
            if v is None:
                if default:
                    return default.strip().strip("'\"")
                raise KeyError(f"environment variable {var} not set (needed by ${{oc.env:{var}}})")
            return v
        if name == "now":
            return _NOW.strftime(arg)
        raise KeyError(f"unknown resolver {name}")
    return _lookup(root, expr)


def _resolve_str(s, root, depth=0):
    """Innermost interpolations first; a string that is (or becomes) exactly one interpolation
    keeps the referenced value's type (so ${eval:'${obs_dim} * ${cond_steps}'} is an int)."""
    if depth > 32:
        raise RecursionError(f"interpolation cycle in {s!r}")

    def rep(mm):
        return str(_resolve_value(_resolver(mm.group(1), root), root, depth + 1))

    out = s
    while True:
        m = _INTERP.fullmatch(out)
        if m:
            return _resolve_value(_resolver(m.group(1), root), root, depth + 1)
        if not _INTERP.search(out):
            return out
        new = _INTERP.sub(rep, out)
        if new == out:
            return out
        out = new


def _resolve_value(v, root, depth=0):
    if isinstance(v, str) and "${" in v:
        return _resolve_str(v, root, depth)
    if isinstance(v, dict):
        return {k: _resolve_value(x, root, depth) for k, x in v.items()}
    if isinstance(v, list):
        return [_resolve_value(x, root, depth) for x in v]
    return v


def resolve(cfg):
    return to_cfg(_resolve_value(to_container(cfg), to_container(cfg)))


def _parse_scalar(s):
    try:
        return yaml.load(s, Loader=_Loader)
    except yaml.YAMLError:
        return s


def apply_overrides(cfg, overrides):
    cfg = to_container(cfg)
    for ov in overrides:
        delete = ov.startswith("~")
        key, _, val = ov.lstrip("+~").partition("=")
        parts = key.split(".")
        node = cfg
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        if delete:
            node.pop(parts[-1], None)
        else:
            node[parts[-1]] = _parse_scalar(val)
    return to_cfg(cfg)


def _merge(base, over):
    out = dict(base)
    for k, v in over.items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def _load_raw(path):
    with open(path) as f:
        raw = yaml.load(f, Loader=_Loader) or {}
    raw.pop("defaults", None)
    raw.pop("hydra", None)
    base = raw.pop("_base_", None)
    if base:  # this repo's cfgs share one base file; reference cfgs have no _base_ and load as-is
        raw = _merge(_load_raw(os.path.join(os.path.dirname(path), base)), raw)
    return raw


def load_config(config_dir, config_name, overrides=()):
    path = os.path.join(config_dir, config_name if config_name.endswith(".yaml") else config_name + ".yaml")
    cfg = apply_overrides(_load_raw(path), overrides)
    return resolve(cfg)


def get_class(target):
    """Map a reference `_target_` (e.g. model.diffusion.diffusion_ppo.PPODiffusion) onto this package."""
    mod, _, name = target.rpartition(".")
    for cand in (f"{PACKAGE}.{mod}", mod):
        try:
            return getattr(importlib.import_module(cand), name)
        except (ImportError, AttributeError):
            continue
    raise ImportError(f"cannot resolve _target_ {target}")


def instantiate(node, **overrides):
    """hydra.utils.instantiate subset: recursive _target_ construction with kwargs = keys."""
    if isinstance(node, list):
        return [instantiate(x) for x in node]
    if not isinstance(node, dict):
        return node
    if "_target_" not in node:
        return Cfg({k: instantiate(v) for k, v in node.items()})
    kwargs = {k: instantiate(v) for k, v in node.items() if k != "_target_"}
    kwargs.update(overrides)
    return get_class(node["_target_"])(**kwargs)


def literal(s):
    try:
        return ast.literal_eval(s)
    except (ValueError, SyntaxError):
        return s
