"""The attention dropout generator's keep mask (``ops/attention.py:
dropout_keep_mask``, the integer-op oracle the GPU tests hold the kernels'
stored keep bits to, bit for bit) on the CPU: rates and correlations."""
def test_keep_mask_statistics():
    """The counter-based generator (one murmur3 state per query, key block
    and lane half, then a xorshift32 chain): keep rate 1 - p_eff, per-row and
    per-column keep rates within sampling noise, no correlation between
    neighbouring keys (same word, next word, next block) or queries."""
    from distributed_compute_pytorch_amd.ops.attention import dropout_keep_mask, dropout_p_effective

    p = 0.1
    m = dropout_keep_mask(2, 3, 512, p, 20261019).float()
    q = 1 - dropout_p_effective(p)
    assert abs(float(m.mean()) - q) < 2e-3
    sd = (q * (1 - q) / 512) ** 0.5
    assert float(m.mean(-1).std()) < 1.3 * sd and float(m.mean(-2).std()) < 1.3 * sd

    def corr(a, b):
        a, b = a - a.mean(), b - b.mean()
        return float((a * b).mean() / (a.std() * b.std()))

    for d in (1, 4, 8, 32, 64):
        assert abs(corr(m[..., :-d], m[..., d:])) < 0.01, d
    assert abs(corr(m[:, :, :-1], m[:, :, 1:])) < 0.01
