"""The examples run end to end on the CPU tier (tiny shapes): ImageNet training with validation,
checkpoint and resume; DCGAN's three independently scaled losses with checkpoints; the simple
amp + DDP loop over gloo (reference examples/, which ship without tests)."""
import os
import runpy
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _clean_amp():
    from apex.amp._amp_state import _amp_state

    yield
    _amp_state.loss_scalers = []
    h = getattr(_amp_state, "handle", None)
    if h is not None:
        h._deactivate()
        _amp_state.handle = None


def test_imagenet_example_train_validate_checkpoint_resume(tmp_path, capsys):
    ns = runpy.run_path(os.path.join(ROOT, "examples", "imagenet", "main_amp.py"), run_name="example")
    common = ["synthetic", "-a", "resnet18", "-b", "4", "--image-size", "64", "--iters-per-epoch", "2",
              "--val-iters", "1", "-j", "0", "--print-freq", "1", "--checkpoint-dir", str(tmp_path), "--seed", "3"]
    ns["main"](common + ["--epochs", "1"])
    out = capsys.readouterr().out
    assert "Prec@1" in out and "Speed" in out
    ck = tmp_path / "checkpoint.pth.tar"
    assert ck.exists()
    state = torch.load(ck, weights_only=True)
    assert state["epoch"] == 1 and "amp" in state and "loss_scaler0" in state["amp"]
    ns["main"](common + ["--epochs", "2", "--resume", str(ck)])
    out = capsys.readouterr().out
    assert "loaded checkpoint" in out and "Epoch: [1]" in out and "Epoch: [0]" not in out
    assert torch.load(ck, weights_only=True)["epoch"] == 2
    ns["main"](common + ["--evaluate", "--resume", str(ck)])
    assert " * Prec@1" in capsys.readouterr().out


def test_imagenet_lr_schedule():
    ns = runpy.run_path(os.path.join(ROOT, "examples", "imagenet", "main_amp.py"), run_name="example")
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0)
    f = ns["adjust_learning_rate"]
    assert abs(f(opt, 0.4, 0, 0, 100) - 0.4 / 500) < 1e-12  # warmup start
    assert abs(f(opt, 0.4, 10, 0, 100) - 0.4) < 1e-12
    assert abs(f(opt, 0.4, 35, 0, 100) - 0.04) < 1e-12
    assert abs(f(opt, 0.4, 85, 0, 100) - 0.4 * 1e-3) < 1e-12


def test_dcgan_example(tmp_path):
    ns = runpy.run_path(os.path.join(ROOT, "examples", "dcgan", "main_amp.py"), run_name="example")
    d, g = ns["main"](["--batch-size", "2", "--iters", "2", "--ngf", "8", "--ndf", "8", "--nz", "16", "--cpu",
                       "--opt-level", "O0", "--outf", str(tmp_path), "--manualSeed", "1"])
    assert d == d and g == g  # finite
    assert (tmp_path / "netG_epoch_0.pth").exists() and (tmp_path / "fake_samples_epoch_000.npy").exists()
    ns["main"](["--batch-size", "2", "--iters", "1", "--ngf", "8", "--ndf", "8", "--nz", "16", "--cpu",
                "--opt-level", "O0", "--netG", str(tmp_path / "netG_epoch_0.pth"),
                "--netD", str(tmp_path / "netD_epoch_0.pth")])


def _free_port():
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_simple_ddp_example_gloo():
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "examples", "simple", "distributed", "distributed_data_parallel.py"),
                        "--cpu", "--steps", "20"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "final loss" in r.stdout
