"""Generate PyWavelets golden vectors for the 3D DWT / IDWT (pins the ptwt restatement).

Run with the interpreter that has PyWavelets (this container: /opt/conda/bin/python3.9,
PyWavelets 1.1.1, numpy 1.26):

    /opt/conda/bin/python3.9 tests/golden/gen_pywt_vectors.py

ptwt 0.1.9 (the reference's un-vendored dependency, requirements.txt:45) implements
wavedec3/waverec3 on top of PyWavelets' filter banks and is tested against
pywt.wavedecn/waverecn(mode='zero', axes=(-3,-2,-1)); these vectors are that contract.
Writes tests/golden/pywt_dwt3.npz.
"""
import os

import numpy as np
import pywt

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rs = np.random.RandomState(1234)
    out = {}
    cases = [
        ("haar", (2, 2, 8, 8, 8), 3),
        ("haar", (1, 2, 4, 6, 10), 2),
        ("db2", (1, 2, 12, 12, 12), 2),
        ("db2", (1, 1, 11, 9, 7), 2),
        ("db3", (1, 2, 13, 10, 17), 2),
        ("db4", (1, 1, 20, 19, 9), 2),
    ]
    for ci, (wav, shape, levels) in enumerate(cases):
        x = rs.standard_normal(shape)
        out[f"c{ci}_x"] = x
        out[f"c{ci}_meta"] = np.array([levels], dtype=np.int64)
        out[f"c{ci}_wavelet"] = np.frombuffer(wav.encode(), dtype=np.uint8)
        for L in range(1, levels + 1):
            coeffs = pywt.wavedecn(x, wav, mode="zero", level=L, axes=(-3, -2, -1))
            out[f"c{ci}_L{L}_ll"] = coeffs[0]
            for li, d in enumerate(coeffs[1:]):  # coarse -> fine
                for k, v in d.items():
                    out[f"c{ci}_L{L}_d{li}_{k}"] = v
            out[f"c{ci}_L{L}_rec"] = pywt.waverecn(coeffs, wav, mode="zero", axes=(-3, -2, -1))
    np.savez_compressed(os.path.join(HERE, "pywt_dwt3.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
