"""The Keras-3 `.weights.h5` boundary: util/h5.py against files written
by a real HDF5 library, its writer against a real HDF5 reader, and the reference models' Keras
layouts (util/keras_weights.py)."""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

from diffusionpolicyoptimization_amd.util import keras_weights as KW
from diffusionpolicyoptimization_amd.util.h5 import H5FormatError, read_h5, write_h5

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from h5_fixture_spec import CH, HIDDEN, fixture_arrays  # noqa: E402

H5PY_PYTHON = "/opt/conda/bin/python3.9"


def _same(want, got):
    bad = [k for k in want if k not in got or np.asarray(want[k]).dtype != got[k].dtype
           or np.shape(want[k]) != got[k].shape or not np.array_equal(np.asarray(want[k]), got[k])]
    assert not bad, bad


@pytest.mark.parametrize("name,many", [("keras_weights_h5py.weights.h5", True),
                                       ("keras_weights_h5py_latest.weights.h5", False)],
                         ids=["h5py-default", "h5py-libver-latest"])
def test_reader_reads_files_written_by_hdf5(name, many):
    """h5py default (superblock v0, symbol tables, a 12-child group over two symbol-table nodes) and
    libver latest (superblock v3, v2 object headers, link messages, layout v4)."""
    arrays, groups = fixture_arrays(many)
    got = read_h5(os.path.join(GOLDEN, name))
    g = got.pop("__groups__")
    assert set(got) == set(arrays)
    _same(arrays, got)
    assert "extra/empty" in g and "actor/vars" in g


def test_writer_round_trip(tmp_path):
    arrays, groups = fixture_arrays()
    p = str(tmp_path / "w.weights.h5")
    write_h5(p, arrays, groups)
    got = read_h5(p)
    assert "extra/empty" in got.pop("__groups__")
    _same(arrays, got)


@pytest.mark.skipif(not os.path.exists(H5PY_PYTHON), reason="no interpreter with h5py in this image")
def test_writer_output_opens_in_h5py(tmp_path):
    arrays, groups = fixture_arrays()
    p = str(tmp_path / "w.weights.h5")
    write_h5(p, arrays, groups)
    r = subprocess.run([H5PY_PYTHON, os.path.join(GOLDEN, "h5py_dump.py"), p], capture_output=True, text=True,
                       timeout=120)
    if r.returncode != 0 and "No module named 'h5py'" in r.stderr:
        pytest.skip("h5py not importable")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout)
    for k, v in arrays.items():
        a = np.asarray(v)
        assert d[k][0] == str(a.dtype) and d[k][1] == list(a.shape), (k, d[k])
        assert abs(d[k][2] - float(a.astype(np.float64).sum())) <= 1e-9 * (1 + abs(d[k][2])), k
    assert "extra/empty/" in d


def test_reader_rejects_non_hdf5(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file" * 10)
    with pytest.raises(H5FormatError):
        read_h5(str(p))


def _specs():
    from diffusionpolicyoptimization_amd import ops
    d = ops.ModelDims(actor_hidden=HIDDEN, critic_hidden=CH)
    return ops.actor_param_spec(d), ops.critic_param_spec(d)


def test_keras_layout_of_a_ppo_checkpoint():
    """load_ppo_model maps actor/, actor_ft/ and critic/ of a PPODiffusion.save_weights file (the
    h5py-written fixture) onto the flat specs; load_actor finds the network inside it too."""
    a_spec, c_spec = _specs()
    arrays, _ = fixture_arrays()
    w = KW.load_ppo_model(os.path.join(GOLDEN, "keras_weights_h5py.weights.h5"), a_spec, c_spec)
    for key, paths in (("actor", KW.actor_paths("actor/")), ("actor_ft", KW.actor_paths("actor_ft/")),
                       ("critic", KW.critic_paths("critic/"))):
        for n, path in paths.items():
            np.testing.assert_array_equal(w[key][n], arrays[path])
    net = KW.load_actor(os.path.join(GOLDEN, "keras_weights_h5py.weights.h5"), a_spec)
    np.testing.assert_array_equal(net["in_w"], arrays["actor/mlp_mean/input_layer/vars/0"])


def test_keras_layout_round_trip_and_errors(tmp_path):
    a_spec, c_spec = _specs()
    rng = np.random.default_rng(0)
    mk = lambda spec: {n: rng.standard_normal(s).astype(np.float32) for n, s in spec}
    actor, ft, critic = mk(a_spec), mk(a_spec), mk(c_spec)
    p = str(tmp_path / "state_3.weights.h5")
    KW.save_ppo_model(p, actor, ft, critic)
    w = KW.load_ppo_model(p, a_spec, c_spec)
    for key, ref in (("actor", actor), ("actor_ft", ft), ("critic", critic)):
        for n in ref:
            np.testing.assert_array_equal(w[key][n], ref[n])
    # a pretrain checkpoint: the network at the root; container names matched by structure
    q = str(tmp_path / "net.weights.h5")
    KW.save_actor(q, actor)
    np.testing.assert_array_equal(KW.load_actor(q, a_spec)["l2_w"], actor["l2_w"])
    d = read_h5(q)
    d.pop("__groups__")
    ren = {k.replace("two_layer_pre_activation_res_net_linear", "block_x")
            .replace("layers/dense_1/", "layers/dense_7/").replace("layers/dense/", "layers/dense_3/"): v
           for k, v in d.items()}
    r = str(tmp_path / "renamed.weights.h5")
    write_h5(r, ren)
    got = KW.load_actor(r, a_spec)
    for n in actor:
        np.testing.assert_array_equal(got[n], actor[n])
    # wrong width -> a clear shape error; missing layer -> named
    from diffusionpolicyoptimization_amd import ops
    big = ops.actor_param_spec(ops.ModelDims(actor_hidden=512))
    with pytest.raises(ValueError, match="shape"):
        KW.load_actor(q, big)
    del ren["mlp_mean/output_layer/vars/0"]
    write_h5(r, ren)
    with pytest.raises(ValueError, match="output_layer"):
        KW.load_actor(r, a_spec)


def test_keras_reader_fails_loudly_on_unmapped_variables(tmp_path):
    """A Keras file with a variable inside the model that the layout does not map (a renamed or
    extra layer) must not load with it silently skipped; state outside the model is only logged."""
    a_spec, c_spec = _specs()
    rng = np.random.default_rng(1)
    mk = lambda spec: {n: rng.standard_normal(s).astype(np.float32) for n, s in spec}
    p = str(tmp_path / "state_1.weights.h5")
    KW.save_ppo_model(p, mk(a_spec), mk(a_spec), mk(c_spec))
    d = read_h5(p)
    d.pop("__groups__")
    d["optimizer/vars/0"] = np.zeros(3, np.float32)          # outside the model: tolerated (logged)
    q = str(tmp_path / "extra_ok.weights.h5")
    write_h5(q, d)
    KW.load_ppo_model(q, a_spec, c_spec)
    d["actor_ft/mlp_mean/extra_layer/vars/0"] = np.zeros((4, 4), np.float32)   # inside: fails, named
    r = str(tmp_path / "extra_bad.weights.h5")
    write_h5(r, d)
    with pytest.raises(ValueError, match="extra_layer"):
        KW.load_ppo_model(r, a_spec, c_spec)
    with pytest.raises(ValueError, match="extra_layer"):
        KW.load_actor(r, a_spec, prefixes=("actor_ft/",))


def test_ppo_checkpoint_carries_learnable_eta(tmp_path):
    """A learn_eta model's checkpoint holds the eta logit (eta/vars/0, where Keras 3 writes a
    sub-layer's variable) and its optimizer state; a model without it has no eta group."""
    import numpy as np
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util import keras_weights as K
    d = ops.ModelDims()
    a, c = ops.actor_param_spec(d), ops.critic_param_spec(d)
    rng = np.random.default_rng(0)
    A = {n: rng.normal(size=s).astype(np.float32) for n, s in a}
    C = {n: rng.normal(size=s).astype(np.float32) for n, s in c}
    p = str(tmp_path / "eta.weights.h5")
    K.save_ppo_model(p, A, A, C, eta={"logit": 0.25, "m": 1e-3, "v": 2e-6, "step": 7})
    w = K.load_ppo_model(p, a, c)
    assert w["eta"] == {"logit": 0.25, "m": 1e-3, "v": 2e-6, "step": 7}
    np.testing.assert_array_equal(w["critic"]["l1_w"], C["l1_w"])
    q = str(tmp_path / "plain.weights.h5")
    K.save_ppo_model(q, A, A, C)
    assert "eta" not in K.load_ppo_model(q, a, c)
