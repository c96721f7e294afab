"""Cooperative recurrences fail loudly (coop.h).

The cooperative kernels (lstm_coop.hip, ardec.hip) split one recurrence over many workgroups
that hand h / dG to each other every step, so every workgroup of a 32-sequence tile must be
resident at once.  When one never arrives (here: the test switch ensvs_coop_inject_fault makes
workgroup 0 skip its step-1 signal) the polls time out, the launch ends within one timeout
(not one per step), and the failure reaches the product:

* the tile's header flag and the process's persistent error word are set;
* the training step's gradient norm is NaN, so the update is skipped (parameters, Adam moments
  and the device step counter unchanged) -- the step does not apply the garbage gradients;
* the host raises engine.CoopError from step_metrics and from the next train_step, and the
  flag is cleared so training can go on;
* the step's gradient norm snapshots and clears the live word, so a step enqueued after the
  failed one (before the host noticed) applies its own update.
"""
import math
import time

import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, data, engine, train
from ensemble_svs_with_interactions_amd._lib import call, query
from ensemble_svs_with_interactions_amd.train import FusedAdam, step_metrics, train_step

pytestmark = pytest.mark.gpu

TIMEOUT_US = 20000


@pytest.fixture
def fault():
    engine.coop_error_word("cuda").zero_()
    call("ensvs_coop_set_timeout_us", TIMEOUT_US)
    call("ensvs_coop_inject_fault", 1)
    yield
    call("ensvs_coop_inject_fault", 0)
    call("ensvs_coop_set_timeout_us", 1000000)
    engine.coop_error_word("cuda").zero_()


def _lstm_launch(H, B, T):
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(B)
    gx = torch.randn(B * T, 8 * H, device="cuda", generator=g) * 0.3
    whh = [torch.randn(4 * H, H, device="cuda", generator=g) * H ** -0.5 for _ in range(2)]
    lens = torch.full((B,), T, dtype=torch.int64, device="cuda")
    wpf = torch.empty(2 * 4 * H * H, dtype=torch.float16, device="cuda")
    call("ensvs_lstm_coop_pack", whh[0].data_ptr(), whh[1].data_ptr(), H, 0, wpf.data_ptr(), st)
    nbytes = query("ensvs_lstm_coop_work_bytes", H, B)
    work = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    y = torch.empty(B * T, 2 * H, device="cuda")
    saved = torch.empty(B * T * 10 * H, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    call("ensvs_lstm_coop_fwd", gx.data_ptr(), 8 * H, wpf.data_ptr(), lens.data_ptr(), B, T, H,
         y.data_ptr(), 2 * H, saved.data_ptr(), work.data_ptr(), nbytes, st)
    torch.cuda.synchronize()
    flags = [work[2048 * z + 128:2048 * z + 132].cpu().view(torch.int32).item()
             for z in range((B + 31) // 32)]
    return time.time() - t0, flags


def test_coop_timeout_ends_launch_and_sets_flags(fault):
    H, B, T = 256, 40, 512
    word = engine.coop_error_word("cuda")
    el, flags = _lstm_launch(H, B, T)
    # one timeout for the whole launch (512 steps would take >= 10 s at one per step)
    assert el < 2.0, el
    assert flags[0] == 1 and flags[1] == 0  # tile 0 failed, tile 1 ran normally
    assert int(word[0].item()) == 1 and int(word[1].item()) == 0  # live word, no step yet
    with pytest.raises(engine.CoopError):
        engine.check_coop_errors("cuda")
    assert int(word.max().item()) == 0  # cleared by the raise
    call("ensvs_coop_inject_fault", 0)
    el, flags = _lstm_launch(H, B, T)
    assert flags == [0, 0] and int(word.max().item()) == 0
    engine.check_coop_errors("cuda")


def _setup(P=4, T=64):
    engine.set_gemm_precision("bf16")
    torch.manual_seed(0)
    m = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).cuda()
    b = data.synthetic_batch(P, T, 5)
    g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
    args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
            b["lengths"].tolist())
    return m, FusedAdam(m), args


def test_train_step_skips_update_and_raises(fault):
    m, opt, args = _setup()
    before = opt.flat.clone()
    loss, norm = train_step(m, opt, *args)
    torch.cuda.synchronize()
    # the cooperative AR decoder of the lf0 branch hit the fault: flagged, update skipped;
    # the norm moved the live word into the failed-step count
    word = engine.coop_error_word("cuda")
    assert int(word[0].item()) == 0 and int(word[1].item()) == 1
    assert not math.isfinite(norm.item())
    assert torch.equal(opt.flat, before)
    assert opt.device_step == 0 and float(opt.m.abs().max()) == 0.0
    with pytest.raises(engine.CoopError):
        step_metrics(loss, opt)
    call("ensvs_coop_inject_fault", 0)
    loss, norm = train_step(m, opt, *args)
    metrics = step_metrics(loss, opt)
    assert math.isfinite(metrics["GradNorm"])
    assert opt.device_step == 1 and not torch.equal(opt.flat, before)


def test_next_train_step_raises(fault):
    m, opt, args = _setup()
    train_step(m, opt, *args)
    torch.cuda.synchronize()  # the device has reached the step's flag copy
    with pytest.raises(engine.CoopError):
        train_step(m, opt, *args)
    call("ensvs_coop_inject_fault", 0)
    loss, norm = train_step(m, opt, *args)
    assert math.isfinite(norm.item()) and opt.device_step == 1


def test_step_after_failure_applies_its_update(fault):
    """the host runs ahead of the device, so a step can be enqueued before the host
    sees the previous step's failure.  Only the failed step skips: the next one (fault off)
    applies its update, and the failure is still raised afterwards."""
    m, opt, args = _setup()
    train_step(m, opt, *args)  # faulted: skipped
    call("ensvs_coop_inject_fault", 0)
    # the next step without any host check in between (what train_step does when the device
    # has not reached the failed step's flag copy yet)
    train._loss_and_grads(m, opt, *args, None, True, None, 0.0)
    opt.step()
    torch.cuda.synchronize()
    assert opt.device_step == 1 and math.isfinite(opt.norm.item())
    assert engine.coop_failed("cuda") == 1
    with pytest.raises(engine.CoopError):
        engine.check_coop_errors("cuda")
    assert engine.coop_failed("cuda") == 0
