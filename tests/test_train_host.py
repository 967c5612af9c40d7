"""train.py host logic on CPU: the loss-log line format (util/visualizer.py:215-221), the epoch loop's
schedule — update_learning_rate per epoch, print / save_latest / save_epoch frequencies — against
methods/GAN-based/CycleGANCon/train.py:57-130, with a stand-in model (no GPU work)."""
import os
from collections import OrderedDict

import gbvst.train as T
from gbvst.options import default_opt


class _FakeModel:
    model_names = ["G_A"]

    def __init__(self):
        self.calls = []
        self.step = 0

    def setup(self, opt):
        self.calls.append("setup")

    def update_learning_rate(self):
        self.calls.append("lr")

    def set_input_nhwc(self, *a):
        self.calls.append("in5")

    def set_input_fc2(self, data):
        self.calls.append("in6")

    def optimize_parameters(self, hg=None, hd=None):
        self.step += 1
        self.calls.append("opt")

    def get_current_losses(self):
        return OrderedDict([("D_A", 0.25), ("G_A", 1.0 / 3.0), ("cycle_A", 2.0)])

    def save_networks(self, which):
        self.calls.append("save:%s" % which)


def test_loss_line_format():
    line = T.Visualizer.format_losses(3, 40, OrderedDict([("D_A", 0.25), ("G_A", 1 / 3)]), 0.0123, 0.5)
    assert line == "(epoch: 3, iters: 40, time: 0.012, data: 0.500) D_A: 0.250 G_A: 0.333 "


def test_epoch_loop_schedule(tmp_path):
    opt = default_opt(True, checkpoints_dir=str(tmp_path), name="exp", n_epochs=2, n_epochs_decay=1,
                      batch_size=2, print_freq=4, save_latest_freq=6, save_epoch_freq=2)
    data = [(0, 1, 2, 3, 4)] * 3  # 3 batches of 2 = 6 images per epoch
    m = _FakeModel()
    _, total = T.train(opt, data, model=m, log=lambda *_: None)
    assert total == 18 and m.step == 9
    assert m.calls[0] == "setup" and m.calls.count("lr") == 3
    # save_latest every 6 images (totals 6, 12, 18), save_epoch at epoch 2 ('latest' + '2')
    saves = [c for c in m.calls if c.startswith("save")]
    assert saves == ["save:latest", "save:latest", "save:latest", "save:2", "save:latest"]
    log = open(os.path.join(str(tmp_path), "exp", "loss_log.txt")).read().splitlines()
    assert log[0].startswith("================ Training Loss (")
    # print every 4 images: totals 4, 8, 12, 16 -> 4 lines; epoch_iter restarts per epoch
    body = log[1:]
    assert len(body) == 4
    assert body[0].startswith("(epoch: 1, iters: 4, time: ")
    assert body[1].startswith("(epoch: 2, iters: 2, time: ")
    assert body[0].endswith("D_A: 0.250 G_A: 0.333 cycle_A: 2.000 ")


def test_reference_tuple_input(tmp_path):
    opt = default_opt(True, checkpoints_dir=str(tmp_path), name="e2", n_epochs=1, n_epochs_decay=0,
                      batch_size=1, print_freq=100, save_latest_freq=100, save_epoch_freq=5)
    m = _FakeModel()
    T.train(opt, [(0, 1, 2, 3, 4, 5)], model=m, log=lambda *_: None)
    assert "in6" in m.calls and "in5" not in m.calls


def test_entry_flags():
    syn, rest = T._add_entry_flags(["--synthetic", "8", "--name", "x", "--synthetic=4"])
    assert syn == 4 and rest == ["--name", "x"]


def test_dp_shard_equal_counts():
    """with len % world != 0, every rank must still hold the same item count (DistributedSampler
    drop_last semantics), or the ranks with an extra batch block in the gradient all-reduce."""
    for n in (22208, 22, 7, 3):
        for world in (2, 3, 8):
            shards = [T.shard_indices(n, world, r) for r in range(world)]
            assert len({len(s) for s in shards}) == 1
            flat = sorted(i for s in shards for i in s)
            assert flat == list(range((n // world) * world))


class _MoFake(_FakeModel):
    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None, grad_hook_M=None):
        self.calls.append(("opt", grad_hook_G, grad_hook_D, grad_hook_M))


class _ExtraPhase(_FakeModel):
    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None, grad_hook_X=None):
        pass


def test_dp_hook_reaches_every_phase():
    """MoGAN's motion-net phase (grad_hook_M) gets the DP exchange too; a model with an
    optimizer phase the loop does not know is refused instead of silently diverging."""
    import pytest
    hook = object()
    m = _MoFake()
    T._optimize(m, hook)
    assert m.calls[-1] == ("opt", hook, hook, hook)
    T._optimize(m, None)
    assert m.calls[-1] == ("opt", None, None, None)
    with pytest.raises(NotImplementedError):
        T._optimize(_ExtraPhase(), hook)
    f = _FakeModel()
    T._optimize(f, hook)
    assert f.step == 1


def test_c3_loss_weight_defaults_follow_vgg_source():
    """C3's VGG loss weights: 100 / 500 for the seeded VGG-19, 1 / 0.01 with --vgg_weights (real VGG
    Grams are ~1e4x larger), explicit values kept."""
    from gbvst.cycle_gan_vgg_model import resolve_loss_weights
    from gbvst.options import parse_options
    o = resolve_loss_weights(parse_options(["--model", "cycle_gan_vgg"], True))
    assert (o.lambda_content, o.lambda_style) == (100.0, 500.0)
    o = resolve_loss_weights(parse_options(["--model", "cycle_gan_vgg", "--vgg_weights", "v.pth"], True))
    assert (o.lambda_content, o.lambda_style) == (1.0, 0.01)
    o = resolve_loss_weights(parse_options(["--model", "cycle_gan_vgg", "--vgg_weights", "v.pth",
                                            "--lambda_style", "3"], True))
    assert (o.lambda_content, o.lambda_style) == (1.0, 3.0)


def test_vgg_torchvision_load_is_complete_or_raises():
    """load_torchvision_features maps 'N.*', 'features.N.*' and 'module.features.N.*' keys and
    raises when any conv tensor of the sliced net is missing (a partial or foreign dict must not leave
    the seeded weights under the pretrained loss weights)."""
    import pytest
    import torch
    from gbvst import perceptual
    net = perceptual.Vgg19(seed=3)
    src = perceptual.Vgg19(seed=4)
    sd = {}
    for x, kind, _, _, m in src.layers:
        if kind == "conv":
            sd["module.features.%d.weight" % x] = m.weight.detach().clone()
            sd["module.features.%d.bias" % x] = m.bias.detach().clone() + 0.5
    sd["classifier.0.weight"] = torch.zeros(2, 2)
    net.load_torchvision_features(sd)
    for (x, kind, _, _, m), (_, _, _, _, ms) in zip(net.layers, src.layers):
        if kind == "conv":
            assert torch.equal(m.weight, ms.weight) and torch.equal(m.bias, ms.bias + 0.5)
    part = {k: v for k, v in sd.items() if not k.endswith(".bias")}
    with pytest.raises(KeyError):
        perceptual.Vgg19(seed=3).load_torchvision_features(part)
    with pytest.raises(KeyError):
        perceptual.Vgg19(seed=3).load_torchvision_features({"classifier.0.weight": torch.zeros(2, 2)})
