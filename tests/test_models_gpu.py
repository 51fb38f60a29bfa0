"""End-to-end GPU engine (bf16 NHWC, fused) vs the fp32 CPU engine on whole models."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _randomize_bn(model):
    from bigdl_amd import nn

    g = torch.Generator().manual_seed(3)
    for m in model.flattened_layers():
        if isinstance(m, nn.BatchNormalization) and m.affine:
            m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
            m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)


@pytest.mark.parametrize("depth,dataset,img", [(50, "ImageNet", 224), (20, "CIFAR10", 32)])
def test_resnet_gpu_matches_cpu(depth, dataset, img):
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import ResNet
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(7)
    cpu = ResNet(1000 if dataset == "ImageNet" else 10, depth, dataSet=dataset)
    _randomize_bn(cpu)
    gpu = copy.deepcopy(cpu).to("cuda")
    fuse_for_training(gpu)
    torch.manual_seed(0)
    x = torch.randn(4, 3, img, img)
    nclass = 1000 if dataset == "ImageNet" else 10
    y = torch.randint(1, nclass + 1, (4,)).float()
    crit_c, crit_g = nn.CrossEntropyCriterion(), nn.CrossEntropyCriterion()
    out_c = cpu.forward(x)
    out_g = gpu.forward(x.cuda())
    assert _rel(out_g, out_c) < 5e-2
    lc = crit_c.forward(out_c, y)
    lg = crit_g.forward(out_g, y.cuda())
    assert abs(float(lc) - float(lg)) < 5e-2 * max(1.0, abs(float(lc)))
    cpu.backward(x, crit_c.backward(out_c, y))
    gpu.backward(x.cuda(), crit_g.backward(out_g, y.cuda()))
    _, gc = cpu.parameters()
    _, gg = gpu.parameters()
    fc = torch.cat([t.reshape(-1) for t in gc])
    fg = torch.cat([t.float().cpu().reshape(-1) for t in gg])
    assert _rel(fg, fc) < 1e-1
    # running statistics updated identically
    bn_c = [m for m in cpu.flattened_layers() if isinstance(m, nn.BatchNormalization)]
    bn_g = [m for m in gpu.flattened_layers() if isinstance(m, nn.BatchNormalization)]
    assert _rel(bn_g[0].runningMean, bn_c[0].runningMean) < 5e-2


def test_train_step_gpu_decreases_loss():
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep

    model = ResNet(10, 20, dataSet=DatasetType.CIFAR10)
    st = TrainStep(model, nn.CrossEntropyCriterion(), SGD(0.05, momentum=0.9, dampening=0.0), device="cuda")
    torch.manual_seed(1)
    x = torch.randn(32, 3, 32, 32, device="cuda")
    y = torch.randint(1, 11, (32,), device="cuda").float()
    losses = [float(st.step(x, y)) for _ in range(30)]
    assert losses[-1] < losses[0] * 0.5, losses


def test_lenet_gpu_matches_cpu():
    from bigdl_amd import nn
    from bigdl_amd.models.lenet import LeNet5

    cpu = LeNet5(10)
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(8, 28 * 28)
    y = torch.randint(1, 11, (8,)).float()
    oc, og = cpu.forward(x), gpu.forward(x.cuda())
    assert _rel(og, oc) < 5e-2
    c1, c2 = nn.ClassNLLCriterion(), nn.ClassNLLCriterion()
    c1.forward(oc, y)
    c2.forward(og, y.cuda())
    cpu.backward(x, c1.backward(oc, y))
    gpu.backward(x.cuda(), c2.backward(og, y.cuda()))
    fc = torch.cat([t.reshape(-1) for t in cpu.parameters()[1]])
    fg = torch.cat([t.float().cpu().reshape(-1) for t in gpu.parameters()[1]])
    assert _rel(fg, fc) < 5e-2
