"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the WaveFormer hot path.

`oracle.ref_waveformer` restates the reference algorithm (network_models/*.py of
mahfuzalhasan/WaveFormer, plus the ptwt 0.1.9 wavelet transform it calls) as plain functional
PyTorch on the CPU, including the reference's arithmetic quirks Q1-Q6.  It is the checker that
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg compare the HIP path against;
the product (`waveformer_amd`) never imports anything from here.

Pinning: the wavelet restatement is pinned by PyWavelets 1.1.1 golden vectors and the model
restatement by fixtures produced by running the reference itself in this container
(tests/golden/, generator scripts alongside).
"""
