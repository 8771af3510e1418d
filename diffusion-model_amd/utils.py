"""Drop-in ``utils.Utils`` — the checkpoint and output contract of the sampling
path (reference utils.py:63-73, 216-224).  Training bookkeeping (loss plots,
result records) is out of scope."""
from __future__ import annotations

import os

import torch
from torch import nn


class Utils:
    @staticmethod
    def saveModelParameter(dir_path: str, model: nn.Module) -> None:
        torch.save(model.state_dict(), os.path.join(dir_path, "trained_para.pth"))

    @staticmethod
    def loadModel(path: str, model: nn.Module, device="cpu") -> nn.Module:
        """state_dict load (weights_only) -> strict load_state_dict -> .to(device) -> .eval()."""
        model.load_state_dict(torch.load(path, map_location=device, weights_only=True))
        model.to(device=device)
        model.eval()
        return model

    @staticmethod
    def saveImages(dir_path: str, images) -> None:
        """pic{i+1}.png per image."""
        for i, image in enumerate(images):
            image.save(os.path.join(dir_path, f"pic{i + 1}.png"))
