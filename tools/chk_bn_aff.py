import torch
from bigdl_amd import nn
from bigdl_amd.models.resnet import ResNet, DatasetType
from bigdl_amd.optim.sgd import SGD
from bigdl_amd.optim.train_step import TrainStep
m = ResNet(1000, 50, dataSet=DatasetType.ImageNet)
step = TrainStep(m, nn.CrossEntropyCriterion(), SGD(learningRate=0.1, momentum=0.9), device=torch.device("cuda"))
x = torch.randn(8, 3, 224, 224, device="cuda"); y = torch.randint(1, 1001, (8,), device="cuda").float()
step.step(x, y); torch.cuda.synchronize()
bns = [l for l in m.flattened_layers() if type(l).__name__ == "SpatialBatchNormalization"]
print("BN", len(bns), "fuse_relu", sum(l.fuse_relu for l in bns), "aff", sum(getattr(l, "_aff", None) is not None for l in bns))
