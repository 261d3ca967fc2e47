"""Synthetic, HBM-resident input: one random batch allocated once on the
device; optional per-step label permutation.  Used by bench.py and --synthetic_data trainers."""
import torch


class SyntheticImages:
    def __init__(self, batch_size, height, width, channels=3, num_classes=1000, device="cpu", dtype=None,
                 seed=0, label_offset=0, shuffle_labels=False):
        g = torch.Generator(device="cpu").manual_seed(seed)
        dtype = dtype or (torch.bfloat16 if torch.device(device).type == "cuda" else torch.float32)
        self.images = torch.randn(batch_size, height, width, channels, generator=g).to(device=device, dtype=dtype)
        self.labels = torch.randint(label_offset, num_classes + label_offset, (batch_size,), generator=g).to(device)
        self.shuffle_labels = shuffle_labels
        self.batch_size = batch_size

    def next_batch(self, batch_size=None):
        if self.shuffle_labels:
            self.labels = self.labels[torch.randperm(self.labels.numel(), device=self.labels.device)]
        if batch_size is not None and batch_size != self.batch_size:
            return self.images[:batch_size], self.labels[:batch_size]
        return self.images, self.labels

    def __iter__(self):
        while True:
            yield self.next_batch()


def synthetic_mnist(batch_size, device="cpu", seed=0):
    """BASELINE config #1: LeNet-5 on synthetic MNIST (28x28x1, 10 classes).  Labels are a fixed
    function of the image (sign pattern of quadrant means) so the loss can actually decrease."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = 0.3 * torch.randn(batch_size, 28, 28, 1, generator=g)
    q = torch.stack([x[:, :14, :14].mean((1, 2, 3)), x[:, :14, 14:].mean((1, 2, 3)),
                     x[:, 14:, :14].mean((1, 2, 3))], 1)
    y = ((q > 0).long() * torch.tensor([1, 2, 4])).sum(1) % 10
    return x.to(device), y.to(device)
