"""A reference-contract ``loss_fn`` ported nearly verbatim (data_paral.py:171-189)
runs through ``util.accum_grads`` (loop, scan, full batch) and its gradient --
taken by autograd through ``model.apply`` on the HIP kernels (GPU) or the torch
reference ops (CPU) -- matches the float64 oracle (VERDICT r1 missing #2)."""
import pytest
import torch

import util
from util import Batch, TrainState, accum_grads, fold_rng_over_axis, softmax_cross_entropy_with_integer_labels
from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.ops.kernels import dropout_mask
from jax_distributed_tuts_amd.utils import rng as R
from jax_distributed_tuts_amd.utils.flat import FlatParams

from .oracle import check_grad, mlp_grads_fp64

DATA_AXIS = "data"  # CONFIG.data_axis_name


# --- the reference's loss_fn, jnp/optax calls swapped for their torch twins ---------
def loss_fn(params, apply_fn, batch, rng):
    dropout_rng = fold_rng_over_axis(rng, DATA_AXIS)
    logits = apply_fn({"params": params}, batch.inputs, train=True, rngs={"dropout": dropout_rng})

    loss = softmax_cross_entropy_with_integer_labels(logits, batch.labels)

    correct_pred = torch.eq(torch.argmax(logits, dim=-1), batch.labels)

    bs = batch.inputs.shape[0]
    step_metrics = {"loss": (loss.sum(), bs), "accuracy": (correct_pred.sum(), bs)}
    loss = loss.mean()

    return loss, step_metrics
# ---------------------------------------------------------------------------------


def _setup(dev, dropout):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.utils.config import dp_config

    model = Classifier(dropout_rate=dropout)
    P = FlatParams(model.param_specs(), device=dev).init_(69)
    st = TrainState.create(apply_fn=model, params=P, tx=util.adamw(1e-3), rng=R.PRNGKey(69))
    b = synthetic_batch(dp_config(), 70)
    return st, b, Batch(b.inputs.to(dev), b.labels.to(dev))


def _run(dev, n_mb, use_scan, dropout):
    st, b, bd = _setup(dev, dropout)
    before = {k: v.cpu() for k, v in st.params.state_dict().items()}
    key = R.PRNGKey(7)
    grads, metrics = accum_grads(st, bd, key, n_mb, loss_fn, use_scan=use_scan)
    got = {n: (st.params.g(n) * grads.scale).cpu() for n in st.params.names()}
    masks = None
    if dropout:
        mb = 128 // n_mb
        masks = [[dropout_mask(fold_rng_over_axis(k, DATA_AXIS) & 0xFFFFFFFF, 0, (mb, 512), 1 - dropout), None]
                 for k in R.split(key, n_mb)]
    want = mlp_grads_fp64(before, ["input_dense", "output_dense"], b.inputs, b.labels, masks=masks,
                          keep=1 - dropout, n_mb=n_mb)
    for n in want:
        check_grad(got[n], want[n], n)
    assert int(metrics["loss"][1]) == 128 and int(metrics["accuracy"][1]) == 128
    return st, grads, metrics


@pytest.mark.parametrize("n_mb,use_scan", [(4, False), (4, True), (1, False)])
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_reference_loss_fn_cpu(n_mb, use_scan, dropout):
    _run("cpu", n_mb, use_scan, dropout)


@pytest.mark.gpu
@pytest.mark.parametrize("n_mb,use_scan", [(4, False), (4, True), (1, False)])
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_reference_loss_fn_gpu(n_mb, use_scan, dropout):
    _run(torch.device("cuda", 0), n_mb, use_scan, dropout)


def test_reference_train_step_reduces_loss():
    """The reference's train_step_dp body (data_paral.py:193-238, B4 fixed) written
    against the util API: accum_grads -> apply_gradients -> metrics += ."""
    st, _, bd = _setup("cpu", 0.1)
    losses = []
    for _ in range(6):
        rng, step_rng = R.split(st.rng)
        grads, step_metrics = accum_grads(st, bd, step_rng, 4, loss_fn=loss_fn)
        st = st.apply_gradients(grads=grads, rng=rng)
        losses.append(float(step_metrics["loss"][0]) / step_metrics["loss"][1])
    assert losses[-1] < losses[0] and st.step == 6


def _scan_vs_loop(dev):
    """The rolled (captured on GPU) reference-contract step draws the loop's dropout
    masks: scan == loop, gradient and metrics, bit for bit."""
    from jax_distributed_tuts_amd.utils import train_state as TS

    out = []
    for use_scan in (False, True):
        st, _, bd = _setup(dev, 0.1)
        grads, metrics = accum_grads(st, bd, R.PRNGKey(11), 4, loss_fn, use_scan=use_scan)
        out.append((st.params.grad.clone(), float(metrics["loss"][0]), float(metrics["accuracy"][0])))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1:] == out[1][1:]
    return TS.LAST_SCAN_MODE["mode"]


def test_scan_key_folds_match_host_keys():
    keys = R.split(R.PRNGKey(5), 4)
    idx = torch.tensor([3], dtype=torch.int32)
    sk = fold_rng_over_axis(R.ScanKey.from_keys(keys, idx), DATA_AXIS)
    want = [fold_rng_over_axis(k, DATA_AXIS) for k in keys]
    assert sk.keys == want and int(sk.device_seed()) == want[3] & 0xFFFFFFFF
    assert [R._s64(w) for w in want] == sk.dev.tolist()


def test_reference_scan_equals_loop_cpu():
    assert _scan_vs_loop("cpu") == "eager"


@pytest.mark.gpu
def test_reference_scan_equals_loop_gpu_captured():
    assert _scan_vs_loop(torch.device("cuda", 0)) == "graph"


@pytest.mark.gpu
def test_rolled_step_captures_once_over_a_training_loop():
    """A 10-step training loop through util.accum_grads(use_scan=True) (the reference's
    train_step body, a fresh rng every step) captures the minibatch program ONCE and
    replays it every later step -- and every step equals the unrolled loop's
    gradient and metrics bit for bit (same dropout masks: the cached program's device
    key table is refreshed per call)."""
    from jax_distributed_tuts_amd.utils import train_state as TS

    dev = torch.device("cuda", 0)
    runs = []
    for use_scan in (False, True):
        st, _, bd = _setup(dev, 0.1)
        c0 = TS.SCAN_STATS["captures"]
        grads_seen, losses = [], []
        for _ in range(10):
            rng, step_rng = R.split(st.rng)
            grads, m = accum_grads(st, bd, step_rng, 4, loss_fn=loss_fn, use_scan=use_scan)
            grads_seen.append(st.params.grad.clone())
            losses.append((float(m["loss"][0]), float(m["accuracy"][0])))
            st = st.apply_gradients(grads=grads, rng=rng)
        runs.append((grads_seen, losses, TS.SCAN_STATS["captures"] - c0))
    (g_loop, l_loop, c_loop), (g_scan, l_scan, c_scan) = runs
    assert c_loop == 0 and c_scan == 1
    assert l_loop == l_scan
    for a, b in zip(g_loop, g_scan):
        assert torch.equal(a, b)
