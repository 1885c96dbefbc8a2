"""GPU: the library's per-thread contexts and stream handling (include/hnm.h conventions).

* short-lived threads: each thread's hnm_ctx is destroyed when the thread exits, so the
  number of live contexts stays bounded however many threads come and go;
* concurrent callers on separate per-thread contexts get results bitwise equal to serial
  calls;
* one thread alternating torch streams, with a workspace that grows between calls, gets
  bitwise equal results (the ctx queues each new stream behind the old one);
* a two-phase call whose begin succeeded and whose exchange then failed is aborted, and the
  next call on the same ctx succeeds.
"""
import gc
import threading

import numpy as np
import pytest
import torch

from hnm_recommendation_amd import NeuralCF
from hnm_recommendation_amd import _lib
from hnm_recommendation_amd import sharding as S
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
U, I = 8000, 30_000


@pytest.fixture(scope="module")
def model():
    m = NeuralCF(U, I)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v))
                       for k, v in syn.ncf_state_dict(U, I, seed=12, bias_scale=0.05,
                                                      emb_scale=20.0).items()})
    return m.to(DEV).eval()


def _bits(r):
    return r[1].cpu(), r[0].view(torch.int32).cpu()


def test_thread_contexts_are_released(model):
    users = torch.from_numpy(syn.user_batch(U, 64, seed=1)).to(DEV)
    ref = _bits(model.recommend_with_scores(users))
    gc.collect()
    base = _lib.live_contexts(DEV)
    errs = []

    def work():
        try:
            torch.cuda.set_device(0)
            got = _bits(model.recommend_with_scores(users))
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
        except BaseException as e:  # pragma: no cover - reported below
            errs.append(e)

    for _ in range(12):
        t = threading.Thread(target=work)
        t.start()
        t.join()
    gc.collect()
    assert not errs, errs
    assert _lib.live_contexts(DEV) <= base + 1, (base, _lib.live_contexts(DEV))


def test_concurrent_threads_bitwise(model):
    batches = [torch.from_numpy(syn.user_batch(U, 300 + 37 * j, seed=20 + j)).to(DEV)
               for j in range(4)]
    serial = [_bits(model.recommend_with_scores(b)) for b in batches]
    out = [None] * len(batches)
    errs = []
    start = threading.Barrier(len(batches))

    def work(j):
        try:
            torch.cuda.set_device(0)
            start.wait()
            for _ in range(3):
                out[j] = _bits(model.recommend_with_scores(batches[j]))
        except BaseException as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(j,)) for j in range(len(batches))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for j in range(len(batches)):
        assert torch.equal(out[j][0], serial[j][0]) and torch.equal(out[j][1], serial[j][1])


def test_alternating_streams_with_growing_workspace(model):
    sizes = [40, 900, 120, 2500, 64, 4096]
    batches = [torch.from_numpy(syn.user_batch(U, n, seed=40 + n)).to(DEV) for n in sizes]
    ref = [_bits(model.recommend_with_scores(b)) for b in batches]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for j, b in enumerate(batches):
        s = streams[j % 2]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            r = model.recommend_with_scores(b)
        torch.cuda.current_stream().wait_stream(s)
        got.append(_bits(r))
    for a, b in zip(got, ref):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_failed_exchange_aborts_two_phase_call(model):
    users = torch.from_numpy(syn.user_batch(U, 500, seed=3)).to(DEV)
    ref = _bits(model.recommend_with_scores(users))
    sc = S.ncf_shard_topk(model, 0, I, 12)
    lb = sc.begin(users)                 # begin succeeded: the ctx holds its tables
    assert torch.isfinite(lb).all()
    with pytest.raises(ValueError):
        model.recommend_with_scores(users)   # refused while the pair is open
    sc.abort()                           # what ItemShardedRecommender does on an exception
    assert _bits(model.recommend_with_scores(users))[0].equal(ref[0])
    v, i = sc(users)
    assert torch.equal(i.cpu(), ref[0])


def test_prefilter_stats_keeps_current_device():
    """hnm_ctx_prefilter_stats switches to the ctx's device to read its counters and restores
    the caller's current device on exit: a diagnostics read of another GPU must not
    move this thread's later allocations / launches.  Needs 2 GPUs for the cross-device case;
    the same-device read is checked everywhere."""
    torch.cuda.set_device(0)
    _lib.prefilter_stats(torch.device("cuda", 0))
    assert torch.cuda.current_device() == 0
    if torch.cuda.device_count() < 2:
        pytest.skip("cross-device read needs 2 GPUs")
    _lib.prefilter_stats(torch.device("cuda", 1))
    assert torch.cuda.current_device() == 0
    x = torch.empty(4, device="cuda")
    assert x.device.index == 0
