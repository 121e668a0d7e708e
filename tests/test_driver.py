"""Driver parity: ``magic_amd.main.train`` against the reference loops
``11a/main.py:42-133`` and ``8c/main.py:33-94``, with a stub model on CPU (the loop logic
only; the HIP step is covered by the GPU tests and ``test_driver_on_gpu``)."""
import types

import numpy as np
import pytest

from magic_amd.main import TrainingException, train


class StubVAE:
    """Records every call; partial_fit returns scripted costs."""

    def __init__(self, batch_size=4, reciprocal=True, costs=None, dist=2.0):
        self.batch_size = batch_size
        self.config = types.SimpleNamespace(reciprocal=reciprocal)
        self.costs = list(costs or [])
        self.fit_calls = []
        self.pred_calls = []
        self.dist = dist

    def partial_fit(self, X, overlap_areas):
        self.fit_calls.append((X[0, 0], overlap_areas[0]))
        cost = self.costs.pop(0) if self.costs else 10.0
        return cost, 3.0, 1.0, 1.0, 1.0, np.full(self.batch_size, self.dist)

    def get_predictions(self, X, overlap_areas=None):
        self.pred_calls.append((X[0, 0], overlap_areas[0]))
        return np.full(self.batch_size, self.dist)


def batches(B=4):
    """Batch k: images filled with k, labels filled with 100 + k (a paired dequeue)."""
    k = 0
    while True:
        yield np.full((B, 6), float(k)), np.full(B, 100.0 + k)
        k += 1


def test_11a_eval_cadence_paired_and_inverted():
    vae = StubVAE()
    logs = []
    # n_samples 24, B 4 -> 6 steps per epoch; 11 epochs -> evals at epochs 0 and 10, i == 3
    _, hist = train(vae, batches(), 24, training_epochs=11, driver="11a", log=logs.append)
    mses = [h for h in hist if h[0] == "mse"]
    assert [(h[1], h[2]) for h in mses] == [(0, 3), (10, 3)]
    # paired: the eval images and labels come from the same dequeue
    assert all(x + 100 == a for x, a in vae.pred_calls)
    # the eval dequeue is taken right after step i == 3's batch (11a/main.py:94)
    assert vae.pred_calls[0][0] == 4.0
    # predictions inverted (11a/main.py:100): pred = 1/2, labels 104
    assert mses[0][3] == pytest.approx((0.5 - 104.0) ** 2)
    # epoch averages (11a/main.py:121-122): cost / n_samples * batch_size per step
    ep = [h for h in hist if h[0] == "epoch"]
    assert len(ep) == 11
    assert ep[0][2] == pytest.approx(6 * 10.0 * 4 / 24) and ep[0][3] == pytest.approx(3.0)
    assert logs[-1].startswith("Epoch: 10") and "Average cost: 10" in logs[-1]


def test_11a_no_inversion_for_a_non_reciprocal_model():
    vae = StubVAE(reciprocal=False)
    _, hist = train(vae, batches(), 24, training_epochs=1, driver="11a", log=lambda s: None)
    (mse,) = [h for h in hist if h[0] == "mse"]
    assert mse[3] == pytest.approx((2.0 - 104.0) ** 2)


def test_8c_cadence_unpaired_not_inverted():
    vae = StubVAE(batch_size=2)
    logs = []
    # n_samples 100, B 2 -> 50 steps per epoch; evals at i = 0, 24, 48
    _, hist = train(vae, batches(2), 100, training_epochs=6, driver="8c", log=logs.append)
    mses = [h for h in hist if h[0] == "mse"]
    assert [(h[1], h[2]) for h in mses if h[1] == 0] == [(0, 0), (0, 24), (0, 48)]
    assert len(mses) == 18
    # 8c/main.py:67-68: images and labels from two separate dequeues -> mismatched
    assert all(a == x + 1 + 100 for x, a in vae.pred_calls)
    # no inversion (8c/main.py:69-76): pred 2, labels of the NEXT dequeue
    x0, a0 = vae.pred_calls[0]
    assert mses[0][3] == pytest.approx((2.0 - a0) ** 2)
    # "Epoch: 0001 cost= ..." every 5th epoch (8c/main.py:87-89)
    assert [l.split()[1] for l in logs if l.startswith("Epoch")] == ["0001", "0006"]


def test_nan_cost_raises_training_exception():
    vae = StubVAE(costs=[1.0, 2.0, float("nan")])
    with pytest.raises(TrainingException, match="cost=nan"):
        train(vae, batches(), 24, training_epochs=2, log=lambda s: None)
    assert len(vae.fit_calls) == 3


def test_inf_cost_passes_the_guard_like_the_reference():
    """np.isnan(inf) is False (11a/main.py:77): a +inf cost (BCE saturation) does not stop
    the loop by itself; the NaN arrives one step later (tests/test_gpu_r2.py)."""
    vae = StubVAE(costs=[float("inf"), 1.0])
    # the step after the inf still runs; the epoch line's int(avg_cost) then fails exactly
    # as the reference's would (11a/main.py:125: int(inf) -> OverflowError)
    with pytest.raises(OverflowError):
        train(vae, batches(), 8, training_epochs=1, log=lambda s: None)
    assert len(vae.fit_calls) == 2


def test_keyboard_interrupt_is_swallowed():
    vae = StubVAE()

    def gen():
        yield from (b for _, b in zip(range(5), batches()))
        raise KeyboardInterrupt

    out, hist = train(vae, gen(), 24, training_epochs=3, log=lambda s: None)
    assert out is vae and len(vae.fit_calls) == 4  # 4 steps + the eval dequeue at i == 3


def test_sample_latent_space_grid_layout():
    """11a/utils.py:401-422: tile (nx-i-1, j) holds generate(z = (v[j], v[i])); batched calls of
    at most batch_size rows (host logic, a stand-in generate that encodes z in its pixels)."""
    import numpy as np
    from magic_amd.vae import sample_latent_space

    class Fake:
        latent_dimensions = 2
        batch_size = 7
        calls = []

        def generate(self, z):
            z = np.asarray(z)
            assert 1 <= len(z) <= self.batch_size
            self.calls.append(len(z))
            img = np.zeros((len(z), 16), dtype=np.float32)
            img[:, 0] = z[:, 0]
            img[:, 1] = z[:, 1]
            return img

    f = Fake()
    c = sample_latent_space(f, nx=5, ny=5)
    assert c.shape == (20, 20)
    v = np.linspace(-3, 3, 5)
    for i in range(5):
        for j in range(5):
            tile = c[(5 - i - 1) * 4:(5 - i) * 4, j * 4:(j + 1) * 4].reshape(-1)
            assert tile[0] == np.float32(v[j]) and tile[1] == np.float32(v[i])
    assert sum(f.calls) == 25 and max(f.calls) == 7

    # nx != ny: nx tiles tall (z[1] = v[i]), ny tiles wide (z[0] = w[j])
    c = sample_latent_space(Fake(), nx=3, ny=4)
    assert c.shape == (12, 16)
    v, w = np.linspace(-3, 3, 3), np.linspace(-3, 3, 4)
    for i in range(3):
        for j in range(4):
            tile = c[(3 - i - 1) * 4:(3 - i) * 4, j * 4:(j + 1) * 4].reshape(-1)
            assert tile[0] == np.float32(w[j]) and tile[1] == np.float32(v[i])

    class Fake3(Fake):
        latent_dimensions = 3

    assert sample_latent_space(Fake3()) is None
