"""Golden vectors for Predictor.predict_raw_probability (light_training/prediction.py:35-63).

The reference module cannot be imported here (it imports SimpleITK and skimage, absent from
this image), so the vectors restate its resample lines verbatim in behaviour: for every class
channel c, torch.nn.functional.interpolate(model_output[c][None, None], mode="trilinear",
size=(d, w, h))[0, 0] assigned into a torch.half buffer -- run on the CPU with PyTorch
2.10.0 (fp32 arithmetic, round-to-nearest fp16 store).  Cases: down-sampling (BraTS crop to
a smaller spacing grid), up-sampling, mixed per-axis ratios, a singleton axis.

    python tests/golden/gen_resample_fixtures.py   ->  tests/golden/resample_fixtures.npz
"""
import os

import numpy as np
import torch

CASES = {  # name: (C, in (D, H, W), out (d, w, h), seed)
    "down": (4, (24, 20, 18), (17, 13, 11), 1),
    "up": (3, (9, 7, 10), (23, 16, 31), 2),
    "mixed": (4, (16, 11, 30), (21, 11, 19), 3),
    "single": (2, (1, 8, 9), (5, 8, 14), 4),
}


def main():
    out = {}
    for name, (C, src, dst, seed) in CASES.items():
        g = torch.Generator().manual_seed(seed)
        x = torch.softmax(torch.randn((C,) + src, generator=g) * 3, 0)
        ref = torch.zeros((C,) + dst, dtype=torch.half)
        for c in range(C):
            ref[c] = torch.nn.functional.interpolate(x[c][None, None], mode="trilinear",
                                                     size=dst)[0, 0]
        out[name + "_in"] = x.numpy()
        out[name + "_out"] = ref.numpy()
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                     "resample_fixtures.npz"), **out)


if __name__ == "__main__":
    main()
