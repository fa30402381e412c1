"""MNIST MLP (784-512-512-10) and its evaluation loop -- the reference's train_mlp.py
(train_mlp.py:10-26 MNISTMLP, :44-64 test).  Training itself is out of scope."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class MNISTMLP(nn.Module):
    def __init__(self):
        super(MNISTMLP, self).__init__()
        self.features = nn.Sequential(
            nn.Linear(784, 512),
            nn.ReLU(),
            nn.Dropout(0.2),
            nn.Linear(512, 512),
            nn.ReLU(),
            nn.Dropout(0.2),
            nn.Linear(512, 10)
        )

    def forward(self, x):
        x = self.features(x.flatten(1))
        output = F.log_softmax(x, dim=1)
        return output


def test(args, model, device, test_loader, pct=1.0):
    """Accuracy over (pct of) the test set, normalised by the full set size as the
    reference does (train_mlp.py:44-64)."""
    model.eval()
    test_loss = 0
    correct = 0
    eval_samples = round(pct * len(test_loader.dataset.targets))
    curr_samples = 0
    with torch.no_grad():
        for data, target in test_loader:
            curr_samples += len(target)
            data, target = data.to(device), target.to(device)
            output = model(data)
            test_loss += F.nll_loss(output, target, reduction='sum').item()
            pred = output.argmax(dim=1, keepdim=True)
            correct += pred.eq(target.view_as(pred)).sum().item()

            if curr_samples >= eval_samples:
                break

    test_loss /= len(test_loader.dataset)

    return correct / len(test_loader.dataset)
