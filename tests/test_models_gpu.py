"""End-to-end GPU engine (bf16 NHWC, fused) vs the fp32 CPU engine on whole models."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _cos(a, b):
    a, b = a.float().cpu().reshape(-1), b.float().cpu().reshape(-1)
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def _weight_grads(model):
    """Gradients of weights only: a conv bias followed by train-mode BN has ~0 gradient by construction,
    so its relative error is meaningless."""
    from bigdl_amd import nn

    out = []
    for m in model.flattened_layers():
        if m.modules_list() or m.parameters() is None:
            continue
        for (w, g) in m._params:
            if w == "bias" and isinstance(m, nn.SpatialConvolution):
                continue
            t = getattr(m, g, None)
            if t is not None:
                out.append(t.float().cpu().reshape(-1))
    return torch.cat(out)


def _randomize_bn(model):
    from bigdl_amd import nn

    g = torch.Generator().manual_seed(3)
    for m in model.flattened_layers():
        if isinstance(m, nn.BatchNormalization) and m.affine:
            m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
            m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)


@pytest.mark.parametrize("stride,nin,n", [(1, 256, 64), (2, 256, 128), (1, 64, 64)])
def test_bottleneck_block_fused_matches_cpu(stride, nin, n):
    """One fused ResNet bottleneck (conv->BN stats epilogue, BN+ReLU, shortcut-first residual add+ReLU in
    the last BN, phase-decomposed stride-2 dgrad) vs the fp32 CPU engine — tight tolerance."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import _Builder
    from bigdl_amd.nn.fusion import fuse_for_training

    b = _Builder("B", True)
    b.iChannels = nin
    cpu = b.bottleneck(n, stride)
    _randomize_bn(cpu)
    gpu = copy.deepcopy(cpu).to("cuda")
    ref = copy.deepcopy(cpu).to("cuda")     # same bf16 kernels, no fusion plan
    fuse_for_training(gpu)
    assert gpu._residual_plan is not None and ref._residual_plan is None
    torch.manual_seed(0)
    x = torch.randn(8, nin, 16, 16).to(torch.bfloat16).float()
    oc = cpu.forward(x)
    og = gpu.forward(x.cuda())
    orf = ref.forward(x.cuda())
    assert _rel(og, orf) < 1e-2
    assert _rel(og, oc) < 2e-2
    gy = torch.randn_like(oc).to(torch.bfloat16).float()
    gc = cpu.backward(x, gy)
    gg = gpu.backward(x.cuda(), gy.cuda())
    gr = ref.backward(x.cuda(), gy.cuda())
    # fusion changes only rounding points; vs fp32 the ReLU masks of near-zero activations differ, so
    # compare directions (see tools/diag_layers.py for the per-layer analysis)
    assert _rel(gg, gr) < 5e-2
    assert _cos(gg, gc) > 0.97
    fg, fr, fc = _weight_grads(gpu), _weight_grads(ref), _weight_grads(cpu)
    assert _rel(fg, fr) < 5e-2
    assert _cos(fg, fc) > 0.97


def test_bottleneck_masked_residual_addend(monkeypatch):
    """Identity-shortcut block with the masked residual addend (nn.fusion.MASKED_ADDEND: the shortcut gradient
    dz * (y > 0) is never written; the first dgrad GEMM adds dz where the BN sign mask is set) against the dres path:
    same input gradient and weight gradients (up to fp32 atomic order), and the masked path actually ran."""
    from bigdl_amd.models.resnet import _Builder
    from bigdl_amd.nn import fusion
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.ops import conv as cv

    b = _Builder("B", True)
    b.iChannels = 256
    blk = b.bottleneck(64, 1)
    _randomize_bn(blk)
    seen = []
    orig = cv.conv2d_dgrad

    def spy(*a, **k):
        seen.append(k.get("addend_zm") is not None)
        return orig(*a, **k)

    monkeypatch.setattr(cv, "conv2d_dgrad", spy)
    torch.manual_seed(1)
    x = torch.randn(4, 256, 14, 14).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = {}
    saved = fusion.MASKED_ADDEND[0]
    for on in (True, False):
        m = copy.deepcopy(blk).to("cuda")
        fuse_for_training(m)
        fusion.MASKED_ADDEND[0] = on
        try:
            m.forward(x)
            g = m.backward(x, gy)
        finally:
            fusion.MASKED_ADDEND[0] = saved      # restore the default (on), not a fixed value
        res[on] = (g.float().clone(), _weight_grads(m))
    assert any(seen)
    # fp32 atomic order in the BN backward reductions (slotted, scheduling-dependent) flips isolated bf16 roundings
    assert _rel(res[True][0], res[False][0]) < 1e-4
    assert _rel(res[True][1], res[False][1]) < 1e-4
    # and against the fp32 engine on the CPU (same bf16-rounded input / gradient): only rounding points differ
    cpu = copy.deepcopy(blk)
    xc, gyc = x.float().cpu().contiguous(), gy.float().cpu().contiguous()
    cpu.forward(xc)
    gc = cpu.backward(xc, gyc)
    # (bf16 activations through three convs and three BNs with batch-4 statistics: ~7 % relative, direction kept)
    assert _rel(res[True][0], gc) < 0.1
    assert _cos(res[True][0], gc) > 0.98
    assert _cos(res[True][1], _weight_grads(cpu)) > 0.98


@pytest.mark.parametrize("depth,dataset,img", [(50, "ImageNet", 224), (20, "CIFAR10", 32)])
def test_resnet_gpu_matches_cpu(depth, dataset, img):
    """Whole network: bf16 activations through 50 layers with batch-4 BN statistics drift a few percent
    from the fp32 engine; exactness is pinned per block above. Uses the builder's own init: with randomized
    BN gammas the 50-layer gradient is chaotic — fp32 vs fp32-with-bf16-rounded-inputs alone gives cosine 0.3."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import ResNet
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(7)
    cpu = ResNet(1000 if dataset == "ImageNet" else 10, depth, dataSet=dataset)
    gpu = copy.deepcopy(cpu).to("cuda")
    fuse_for_training(gpu)
    torch.manual_seed(0)
    x = torch.randn(4, 3, img, img)
    nclass = 1000 if dataset == "ImageNet" else 10
    y = torch.randint(1, nclass + 1, (4,)).float()
    crit_c, crit_g = nn.CrossEntropyCriterion(), nn.CrossEntropyCriterion()
    out_c = cpu.forward(x)
    out_g = gpu.forward(x.cuda())
    tol = 0.2 if depth >= 50 else 5e-2
    assert _rel(out_g, out_c) < tol
    lc = crit_c.forward(out_c, y)
    lg = crit_g.forward(out_g, y.cuda())
    assert abs(float(lc) - float(lg)) < tol * max(1.0, abs(float(lc)))
    cpu.backward(x, crit_c.backward(out_c, y))
    gpu.backward(x.cuda(), crit_g.backward(out_g, y.cuda()))
    fc, fg = _weight_grads(cpu), _weight_grads(gpu)
    assert _cos(fg, fc) > 0.9
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
    # the training step runs on a high-priority compute stream (ops/side_stream.py priority_compute_stream): the
    # weight-gradient side stream stays at normal priority
    from bigdl_amd.ops import side_stream

    assert torch.cuda.current_stream().priority < 0
    ss = side_stream.stream_for(x)
    assert ss is not None and ss.priority == 0


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


@pytest.mark.parametrize("name,shape", [("VggForCifar10", (4, 3, 32, 32)),
                                        ("Inception_v1_NoAuxClassifier", (2, 3, 224, 224)),
                                        ("Inception_v2_NoAuxClassifier", (2, 3, 224, 224))])
def test_zoo_models_gpu_match_cpu(name, shape):
    """Concat branches, LRN, ceil-mode pooling, BN eps 1e-3 and dropout-free eval on the GPU engine."""
    from bigdl_amd import models as M
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(11)
    cpu = getattr(M, name)(10)
    cpu.evaluate()
    gpu = copy.deepcopy(cpu).to("cuda")
    gpu.evaluate()
    x = torch.randn(*shape)
    assert _rel(gpu.forward(x.cuda()), cpu.forward(x)) < 5e-2


def test_ir_dnn_inference_fusion_matches_cpu():
    """IRToDnn: BN folded into conv weights + ReLU in the conv epilogue on the GPU engine vs the CPU model."""
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.utils.intermediate import ConversionUtils

    torch.manual_seed(0)
    m = ResNet(10, 20, dataSet=DatasetType.CIFAR10)
    for layer in m.flattened_layers():
        if hasattr(layer, "runningMean"):
            layer.runningMean.uniform_(-0.2, 0.2)
            layer.runningVar.uniform_(0.8, 1.2)
    m.evaluate()
    x = torch.randn(8, 3, 32, 32)
    ref = m.forward(x)
    g = ConversionUtils.convert(m, "dnn", device="cuda", train=False)
    out = g.forward(x.cuda()).float().cpu()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel


def test_inception_v3_gpu_matches_cpu():
    """Inception-v3 (factorised 1x7 / 7x1 / 1x3 / 3x1 kernels, avg-pool branches) on the GPU engine vs CPU fp32."""
    from bigdl_amd.models.inception import Inception_v3

    torch.manual_seed(0)
    m = Inception_v3(100)
    m.evaluate()
    x = torch.randn(2, 3, 299, 299)
    ref = m.forward(x)
    g = copy.deepcopy(m).to("cuda")
    out = g.forward(x.cuda()).float().cpu()
    rel = ((out.exp() - ref.exp()).norm() / ref.exp().norm()).item()
    assert rel < 3e-2, rel


def test_dgrad_epilogue_bn_reduction_matches_separate_pass(monkeypatch):
    """Two stacked bottlenecks: the BN backward reductions computed in the consumer conv's dgrad epilogue
    (BN->ReLU->conv inside a branch, and the previous block's last BN through the folded residual dgrad)
    match the separate bn_bwd_reduce pass, and that pass is skipped."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import _Builder
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.ops import native

    b = _Builder("B", True)
    b.iChannels = 64
    cpu = nn.Sequential().add(b.bottleneck(64, 1)).add(b.bottleneck(128, 2))
    _randomize_bn(cpu)
    torch.manual_seed(0)
    x = torch.randn(8, 64, 16, 16).to(torch.bfloat16).float().cuda()
    C_ = native.get()
    real = C_.bn_bwd_reduce
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    monkeypatch.setattr(C_, "bn_bwd_reduce", counting)
    res = {}
    from bigdl_amd.nn import fusion

    for mode in ("0", "1"):
        monkeypatch.setenv("BIGDL_DGRAD_BN", mode)     # fusion on / off (see nn/fusion.py)
        # projection-shortcut BNs reduced by the pass that writes the residual gradient: on / off with the rest
        monkeypatch.setattr(fusion, "SHORTCUT_BN_RED", [mode == "1"])
        m = copy.deepcopy(cpu).to("cuda")
        fuse_for_training(m)
        calls.clear()
        out = m.forward(x)
        gy = torch.randn(out.shape, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).cuda()
        gx = m.backward(x, gy.to(out.dtype))
        torch.cuda.synchronize()
        res[mode] = (gx.float(), _weight_grads(m), len(calls))
    n_bn = sum(isinstance(q, nn.BatchNormalization) for q in cpu.flattened_layers())
    assert res["0"][2] == n_bn
    # fused: 2 branch BNs per block + block 1's last BN (through block 2's folded conv1 dgrad) + both blocks'
    # projection-shortcut BNs (in their block's residual-gradient pass)
    assert res["1"][2] == n_bn - 7
    assert _rel(res["1"][0], res["0"][0]) < 2e-2
    assert _rel(res["1"][1], res["0"][1]) < 2e-2


def test_resnet50_every_layer_matches_fp32_on_its_own_input():
    """Pins every conv and BatchNorm of the full (fused) ResNet-50 training forward: each layer's bf16 GPU output
    is compared with the fp32 CPU layer applied to the SAME (GPU-produced) input, so a systematic per-layer error
    anywhere in the 50-layer network cannot hide behind the loose whole-network tolerance above."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import ResNet
    from bigdl_amd.nn.fusion import fuse_for_training
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(7)
    cpu = ResNet(1000, 50, dataSet="ImageNet")
    gpu = copy.deepcopy(cpu).to("cuda")
    fuse_for_training(gpu)
    resid_bns = {id(m._residual_plan[2]) for m in gpu.flattened_layers()
                 if isinstance(m, nn.Sequential) and getattr(m, "_residual_plan", None)}
    pairs = [(g, c) for g, c in zip(gpu.flattened_layers(), cpu.flattened_layers())
             if isinstance(g, (nn.SpatialConvolution, nn.BatchNormalization)) and id(g) not in resid_bns]
    seen = []
    for g, c in pairs:
        orig = g.updateOutput

        def hook(inp, _g=g, _c=c, _orig=orig):
            from bigdl_amd.ops import bn as bnops

            out = _orig(inp)
            real_in, real_out = bnops.materialize(inp), bnops.materialize(out)   # deferred BN outputs (the stem)
            seen.append((_g, _c, real_in.detach().float().cpu().clone(), real_out.detach().float().cpu().clone()))
            return out
        g.updateOutput = hook
    torch.manual_seed(0)
    gpu.forward(torch.randn(4, 3, 224, 224).cuda())
    for g, _ in pairs:
        del g.updateOutput
    assert len(seen) == len(pairs) >= 60
    worst = 0.0
    for g, c, inp, out in seen:
        c.training()
        with torch.no_grad():
            ref = c.forward(inp.contiguous())
        if getattr(g, "fuse_relu", False):
            ref = torch.relu(ref)
        r = _rel(out, ref)
        worst = max(worst, r)
        assert r < 2e-2, (type(g).__name__, g.getName(), r)
    assert worst < 2e-2
