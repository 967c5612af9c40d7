"""CPU oracle for StarGAN.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): stock-PyTorch CPU (NCHW fp32) restatement of
the reference's StarGAN networks and training iteration, checked against fixtures the reference
itself produced (oracle/gen_golden_stargan.py -> tests/golden/stargan_small.npz), then used as the
checker of the HIP path.

Reference files restated (paths relative to the reference root):
  methods/GAN-based/StarGAN/model.py:7-19    ResidualBlock (conv3x3 -> IN(affine, running) -> ReLU
                                             -> conv3x3 -> IN; x + main(x))
  methods/GAN-based/StarGAN/model.py:22-65   Generator (label replicated + concatenated; conv7x7,
                                             2x conv4x4 s2, repeat_num residual blocks, 2x convT
                                             4x4 s2, conv7x7 -> Tanh)
  methods/GAN-based/StarGAN/model.py:68-88   Discriminator (repeat_num x [conv4x4 s2 + LeakyReLU
                                             0.01], conv1 3x3 -> out_src, conv2 kxk -> out_cls)
  methods/GAN-based/StarGAN/solver.py:187-239 gradient_penalty, label2onehot, classification_loss
  methods/GAN-based/StarGAN/solver.py:298-363 one training iteration (D step every iteration with
                                             the WGAN-GP term, G step every n_critic iterations)
solver.py itself is not importable here (it imports torchvision and the repo's sg2_core package),
so the iteration is restated and pinned by a fixture that runs it over the reference's own
model.py modules.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def _in(c):
    return nn.InstanceNorm2d(c, affine=True, track_running_stats=True)


class RefResidualBlock(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.main = nn.Sequential(nn.Conv2d(dim_in, dim_out, 3, 1, 1, bias=False), _in(dim_out), nn.ReLU(),
                                  nn.Conv2d(dim_out, dim_out, 3, 1, 1, bias=False), _in(dim_out))

    def forward(self, x):
        return x + self.main(x)


class RefGenerator(nn.Module):
    def __init__(self, conv_dim=64, c_dim=5, repeat_num=6):
        super().__init__()
        L = [nn.Conv2d(3 + c_dim, conv_dim, 7, 1, 3, bias=False), _in(conv_dim), nn.ReLU()]
        c = conv_dim
        for _ in range(2):
            L += [nn.Conv2d(c, 2 * c, 4, 2, 1, bias=False), _in(2 * c), nn.ReLU()]
            c *= 2
        L += [RefResidualBlock(c, c) for _ in range(repeat_num)]
        for _ in range(2):
            L += [nn.ConvTranspose2d(c, c // 2, 4, 2, 1, bias=False), _in(c // 2), nn.ReLU()]
            c //= 2
        L += [nn.Conv2d(c, 3, 7, 1, 3, bias=False), nn.Tanh()]
        self.main = nn.Sequential(*L)

    def forward(self, x, c):
        c = c.view(c.size(0), c.size(1), 1, 1).expand(-1, -1, x.size(2), x.size(3))
        return self.main(torch.cat([x, c], dim=1))


class RefDiscriminator(nn.Module):
    def __init__(self, image_size=128, conv_dim=64, c_dim=5, repeat_num=6):
        super().__init__()
        L = [nn.Conv2d(3, conv_dim, 4, 2, 1), nn.LeakyReLU(0.01)]
        c = conv_dim
        for _ in range(1, repeat_num):
            L += [nn.Conv2d(c, 2 * c, 4, 2, 1), nn.LeakyReLU(0.01)]
            c *= 2
        k = int(image_size / np.power(2, repeat_num))
        self.main = nn.Sequential(*L)
        self.conv1 = nn.Conv2d(c, 1, 3, 1, 1, bias=False)
        self.conv2 = nn.Conv2d(c, c_dim, k, bias=False)

    def forward(self, x):
        h = self.main(x)
        out_cls = self.conv2(h)
        return self.conv1(h), out_cls.view(out_cls.size(0), out_cls.size(1))


def label2onehot(labels, dim):
    out = torch.zeros(labels.size(0), dim)
    out[np.arange(labels.size(0)), labels.long()] = 1
    return out


def classification_loss(logit, target, dataset="CelebA"):
    if dataset == "CelebA":
        return F.binary_cross_entropy_with_logits(logit, target, reduction="sum") / logit.size(0)
    return F.cross_entropy(logit, target)


def gradient_penalty(y, x):
    dydx = torch.autograd.grad(outputs=y, inputs=x, grad_outputs=torch.ones_like(y), retain_graph=True,
                               create_graph=True, only_inputs=True)[0]
    dydx = dydx.view(dydx.size(0), -1)
    return torch.mean((torch.sqrt(torch.sum(dydx ** 2, dim=1)) - 1) ** 2)


def d_losses(G, D, x_real, label_org, label_trg, alpha, c_dim, lambda_cls=1.0, lambda_gp=10.0, dataset="CelebA"):
    """solver.py:315-335: (d_loss, parts) of the discriminator step."""
    c_org, c_trg = label2onehot(label_org, c_dim), label2onehot(label_trg, c_dim)
    out_src, out_cls = D(x_real)
    d_loss_real = -torch.mean(out_src)
    d_loss_cls = classification_loss(out_cls, c_org, dataset)
    x_fake = G(x_real, c_trg)
    out_src, _ = D(x_fake.detach())
    d_loss_fake = torch.mean(out_src)
    x_hat = (alpha * x_real.data + (1 - alpha) * x_fake.data).requires_grad_(True)
    out_src, _ = D(x_hat)
    d_loss_gp = gradient_penalty(out_src, x_hat)
    d_loss = d_loss_real + d_loss_fake + lambda_cls * d_loss_cls + lambda_gp * d_loss_gp
    return d_loss, {"D/loss_real": d_loss_real.item(), "D/loss_fake": d_loss_fake.item(),
                    "D/loss_cls": d_loss_cls.item(), "D/loss_gp": d_loss_gp.item()}


def g_losses(G, D, x_real, label_org, label_trg, c_dim, lambda_cls=1.0, lambda_rec=10.0, dataset="CelebA"):
    """solver.py:348-363: (g_loss, parts) of the generator step."""
    c_org, c_trg = label2onehot(label_org, c_dim), label2onehot(label_trg, c_dim)
    x_fake = G(x_real, c_trg)
    out_src, out_cls = D(x_fake)
    g_loss_fake = -torch.mean(out_src)
    g_loss_cls = classification_loss(out_cls, c_trg, dataset)
    x_reconst = G(x_fake, c_org)
    g_loss_rec = torch.mean(torch.abs(x_real - x_reconst))
    g_loss = g_loss_fake + lambda_rec * g_loss_rec + lambda_cls * g_loss_cls
    return g_loss, {"G/loss_fake": g_loss_fake.item(), "G/loss_rec": g_loss_rec.item(),
                    "G/loss_cls": g_loss_cls.item()}


def train_iteration(G, D, g_opt, d_opt, x_real, label_org, label_trg, alpha, i, c_dim, n_critic=5,
                    lambda_cls=1.0, lambda_rec=10.0, lambda_gp=10.0, dataset="CelebA"):
    """solver.py:298-363 with the batch, target labels and GP alphas given."""
    d_loss, loss = d_losses(G, D, x_real, label_org, label_trg, alpha, c_dim, lambda_cls, lambda_gp, dataset)
    g_opt.zero_grad()
    d_opt.zero_grad()
    d_loss.backward()
    d_opt.step()
    if (i + 1) % n_critic == 0:
        g_loss, parts = g_losses(G, D, x_real, label_org, label_trg, c_dim, lambda_cls, lambda_rec, dataset)
        g_opt.zero_grad()
        d_opt.zero_grad()
        g_loss.backward()
        g_opt.step()
        loss.update(parts)
    return loss


LOSS_KEYS = ("D/loss_real", "D/loss_fake", "D/loss_cls", "D/loss_gp", "G/loss_fake", "G/loss_rec", "G/loss_cls")


# ------------------------------------------------------------------- fixture weights (PRNG)
def sg_weights(net, base):
    """Counter-PRNG state_dict by name: conv weights N(0, 1/fan_in), biases N(0, 0.05), IN gamma
    N(1, 0.1), beta N(0, 0.1), running_mean N(0, 0.2), running_var U(0.5, 1.5)."""
    from oracle import prng
    sd = {}
    for k, v in net.state_dict().items():
        shape, s = tuple(v.shape), prng.seed_for(k, base)
        if k.endswith("num_batches_tracked"):
            sd[k] = np.array(0, dtype=np.int64)
        elif k.endswith("running_mean"):
            sd[k] = prng.normal(s, shape, std=0.2)
        elif k.endswith("running_var"):
            sd[k] = prng.uniform_f32(s, shape, 0.5, 1.5)
        elif v.dim() == 1:
            sd[k] = prng.normal(s, shape, std=0.1, mean=1.0 if k.endswith("weight") else 0.0) \
                if _is_norm(net, k) else prng.normal(s, shape, std=0.05)
        else:
            fan_in = v.shape[0] if _is_convT(net, k) else int(np.prod(shape[1:]))
            sd[k] = prng.normal(s, shape, std=(1.0 / fan_in) ** 0.5)
    return sd


def _module_of(net, key):
    return dict(net.named_modules())[key.rsplit(".", 1)[0]]


def _is_norm(net, key):
    return isinstance(_module_of(net, key), nn.InstanceNorm2d) or "InstanceNorm" in type(_module_of(net, key)).__name__


def _is_convT(net, key):
    return "ConvTranspose" in type(_module_of(net, key)).__name__
