"""CPU: the fused Adam's host path (toycrystals_amd.optim.Adam.step) with the library call stubbed — step counts
(per parameter, including parameters skipped in some steps), the per-group step views, the cached argument
table, the version bump, and the state_dict round trip.  The arithmetic itself is the GPU test
(tests/test_gpu_train.py::test_adam_matches_torch_adam)."""
import torch

import toycrystals_amd.optim as O


class _Stub:
    def __init__(self):
        self.calls = []

    def tcx_adam(self, table, n, max_n, lr, b1, b2, eps, wd, step, stream):
        self.calls.append((step, [table[i].p for i in range(n)], n))
        return 0


def _opt(monkeypatch, params):
    stub = _Stub()
    monkeypatch.setattr(O, "lib", lambda: stub)
    monkeypatch.setattr(O, "stream_ptr", lambda d: None)
    opt = O.Adam(params, lr=1e-3)
    for p in params:  # (CPU parameters: the CUDA check runs only when state is created)
        st = opt.state[p]
        st["step"] = torch.tensor(0.0)
        st["exp_avg"] = torch.zeros_like(p)
        st["exp_avg_sq"] = torch.zeros_like(p)
    return opt, stub


def test_step_counts_views_table_and_versions(monkeypatch):
    ps = [torch.nn.Parameter(torch.randn(n)) for n in (5, 7, 3)]
    opt, stub = _opt(monkeypatch, ps)
    for p in ps:
        p.grad = torch.zeros_like(p)
    v0 = [p._version for p in ps]
    opt.step()
    opt.step()
    assert [c[0] for c in stub.calls] == [1, 2] and all(c[2] == 3 for c in stub.calls)
    assert all(p._version > v for p, v in zip(ps, v0))
    assert [float(opt.state[p]["step"]) for p in ps] == [2.0, 2.0, 2.0]
    base = opt.state[ps[0]]["step"]._base
    assert base is not None and all(opt.state[p]["step"]._base is base for p in ps)  # one add per group
    # parameter 1 without a gradient: skipped, its count stays; then counts differ -> one launch per count
    ps[1].grad = None
    opt.step()
    assert stub.calls[-1][0] == 3 and stub.calls[-1][2] == 2
    assert [float(opt.state[p]["step"]) for p in ps] == [3.0, 2.0, 3.0]
    ps[1].grad = torch.zeros_like(ps[1])
    opt.step()
    steps = sorted((c[0], c[2]) for c in stub.calls[-2:])
    assert steps == [(3, 1), (4, 2)]
    assert [float(opt.state[p]["step"]) for p in ps] == [4.0, 3.0, 4.0]


def test_state_dict_round_trip_rebinds_steps(monkeypatch):
    ps = [torch.nn.Parameter(torch.randn(4)) for _ in range(3)]
    opt, stub = _opt(monkeypatch, ps)
    for p in ps:
        p.grad = torch.ones_like(p)
    for _ in range(3):
        opt.step()
    sd = opt.state_dict()
    assert [float(sd["state"][i]["step"]) for i in range(3)] == [3.0, 3.0, 3.0]
    opt2, stub2 = _opt(monkeypatch, ps)
    opt2.load_state_dict(sd)
    opt2.step()
    assert stub2.calls[-1][0] == 4
    assert [float(opt2.state[p]["step"]) for p in ps] == [4.0, 4.0, 4.0]
    assert float(sd["state"][0]["step"]) == 3.0  # the saved dict is not advanced by the new optimiser
