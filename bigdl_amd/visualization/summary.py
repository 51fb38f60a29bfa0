"""Training / validation summaries (S/visualization/Summary.scala:32, TrainSummary.scala:32,
ValidationSummary.scala). Event files land in ``logDir/appName/{train,validation}`` and open in TensorBoard."""
import os

from ..optim.trigger import Trigger
from .tensorboard import FileReader, FileWriter, histogram_summary, scalar_summary


class Summary:
    folder = None

    def __init__(self, logDir, appName):
        self.logDir, self.appName = logDir, appName
        self.writer = FileWriter(self.folder)

    def addScalar(self, tag, value, step):
        self.writer.addSummary(scalar_summary(tag, float(value)), int(step))
        return self

    def addHistogram(self, tag, value, step):
        self.writer.addSummary(histogram_summary(tag, value), int(step))
        return self

    def readScalar(self, tag):
        self.writer.flush()
        return FileReader.readScalar(self.folder, tag)

    def close(self):
        self.writer.close()


class TrainSummary(Summary):
    def __init__(self, logDir, appName):
        self.folder = os.path.join(logDir, appName, "train")
        super().__init__(logDir, appName)
        self.triggers = {"Loss": Trigger.severalIteration(1), "Throughput": Trigger.severalIteration(1)}

    def setSummaryTrigger(self, tag, trigger):
        if tag not in ("LearningRate", "Loss", "Throughput", "Parameters"):
            raise ValueError("TrainSummary: only support LearningRate, Loss, Parameters and Throughput")
        self.triggers[tag] = trigger
        return self

    def getSummaryTrigger(self, tag):
        return self.triggers.get(tag)

    def getScalarTriggers(self):
        return [(k, v) for k, v in self.triggers.items() if k != "Parameters"]


class ValidationSummary(Summary):
    def __init__(self, logDir, appName):
        self.folder = os.path.join(logDir, appName, "validation")
        super().__init__(logDir, appName)
