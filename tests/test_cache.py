"""The decoded-shard cache's bounds and concurrency (CPU; streaming_amd/cache.py):
device and host bytes bounded separately, the bound split over DataLoader workers, the most
recently used shard kept even above the bound (no re-decode per read), and decodes of different
shards running concurrently outside the cache lock."""

import threading
import time

import pytest

from streaming_amd import cache as cache_mod
from streaming_amd.cache import DecodedShardCache


def test_device_and_host_bounds_are_separate():
    c = DecodedShardCache(100, host_limit_bytes=50)
    c.put(1, 'a', 60)
    c.put(2, 'b', 30)
    assert c.resident_bytes == 90 and len(c) == 2
    c.set_host_bytes(2, 40)  # host bytes within their own bound: nothing evicted
    assert len(c) == 2 and c.resident_host_bytes == 40
    c.set_host_bytes(1, 40)  # 80 host bytes > 50: the LRU entry (2) goes
    assert 2 not in c and 1 in c and c.resident_host_bytes == 40
    c.put(3, 'c', 50)  # device 60 + 50 > 100: entry 1 evicted
    assert 1 not in c and c.resident_bytes == 50 and c.resident_host_bytes == 0


def test_most_recent_entry_kept_above_the_bound():
    c = DecodedShardCache(100)
    calls = []

    def make(key):
        def create():
            calls.append(key)
            return f'shard{key}', 250  # larger than the whole bound
        return create

    with pytest.warns(UserWarning, match='exceeds the decoded-shard cache bound'):
        assert c.get_or_create(7, make(7)) == 'shard7'
    for _ in range(5):  # repeated reads of that shard: decoded once
        assert c.get_or_create(7, make(7)) == 'shard7'
    assert calls == [7] and c.misses == 1 and c.hits == 5
    c.get_or_create(8, make(8))  # the next shard replaces it
    assert 7 not in c and 8 in c and len(c) == 1


def test_bound_split_over_dataloader_workers(monkeypatch):
    c = DecodedShardCache(1000)
    assert c.device_limit() == 1000
    monkeypatch.setattr(cache_mod, 'worker_share', lambda: 4)
    assert c.device_limit() == 250
    for k in range(10):
        c.put(k, k, 100)
        assert c.resident_bytes <= 250
    assert len(c) == 2


def test_concurrent_first_touches_overlap():
    c = DecodedShardCache(1 << 20)
    spans = {}

    def make(key):
        def create():
            t0 = time.perf_counter()
            time.sleep(0.3)
            spans[key] = (t0, time.perf_counter())
            return key, 10
        return create

    threads = [threading.Thread(target=c.get_or_create, args=(k, make(k))) for k in (1, 2)]
    for t in threads:
        t.start()
    # a hit on a third, resident shard is served while both decodes run
    c.put(3, 'resident', 10)
    t0 = time.perf_counter()
    assert c.get(3) == 'resident'
    assert time.perf_counter() - t0 < 0.1
    for t in threads:
        t.join()
    (a0, a1), (b0, b1) = spans[1], spans[2]
    assert a0 < b1 and b0 < a1, 'the two decodes did not overlap'


def test_same_key_decoded_once_by_concurrent_callers():
    c = DecodedShardCache(1 << 20)
    calls = []
    gate = threading.Event()

    def create():
        calls.append(1)
        gate.wait(5)
        return 'v', 10

    out = []
    threads = [threading.Thread(target=lambda: out.append(c.get_or_create(5, create)))
               for _ in range(4)]
    for t in threads:
        t.start()
    time.sleep(0.1)
    gate.set()
    for t in threads:
        t.join()
    assert calls == [1] and out == ['v'] * 4


def test_failed_decode_reaches_every_waiter_and_is_not_cached():
    c = DecodedShardCache(1 << 20)

    def create():
        time.sleep(0.1)
        raise FileNotFoundError('gone')

    errors = []

    def run():
        try:
            c.get_or_create(9, create)
        except FileNotFoundError as e:
            errors.append(e)

    threads = [threading.Thread(target=run) for _ in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert len(errors) == 3 and 9 not in c


def test_bound_is_per_device():
    """Readers on two GPUs sharing one cache object (the process-wide default) each get the
    whole bound on their own device: an entry of one device never evicts the other's."""
    c = DecodedShardCache(100)
    c.put(1, 'a', 60, device='cuda:0')
    c.put(2, 'b', 60, device='cuda:1')
    assert 1 in c and 2 in c
    assert c.device_bytes('cuda:0') == 60 and c.device_bytes('cuda:1') == 60
    c.put(3, 'c', 60, device='cuda:0')  # cuda:0 over its bound: only cuda:0's LRU goes
    assert 1 not in c and 2 in c and 3 in c
    assert c.resident_bytes == 120
    made = c.get_or_create(4, lambda: ('d', 30, 'cuda:1'))  # create() may name its device
    assert made == 'd' and c.device_bytes('cuda:1') == 90 and 2 in c


def test_limit_zero_keeps_the_last_shard_per_device():
    c = DecodedShardCache(0)
    with pytest.warns(UserWarning):
        c.put(1, 'a', 10, device='cuda:0')
    c.put(2, 'b', 10, device='cuda:0')
    c.put(3, 'c', 10, device='cuda:1')
    assert list(c._entries) == [2, 3]


@pytest.mark.parametrize('how', ['clear', 'discard'])
def test_clear_or_discard_cancels_a_decode_in_flight(how):
    """A decode running while clear() / discard(key) runs is handed to its waiters but not
    inserted: clear() leaves the cache empty."""
    c = DecodedShardCache(1 << 20)
    started, release = threading.Event(), threading.Event()

    def create():
        started.set()
        release.wait(5)
        return 'v', 10

    got = []
    t = threading.Thread(target=lambda: got.append(c.get_or_create(1, create)))
    t.start()
    started.wait(5)
    waiter = threading.Thread(target=lambda: got.append(c.get_or_create(1, lambda: ('x', 1))))
    waiter.start()
    time.sleep(0.05)
    c.clear() if how == 'clear' else c.discard(1)
    release.set()
    t.join(5)
    waiter.join(5)
    assert got == ['v', 'v']
    assert len(c) == 0 and c.resident_bytes == 0
    assert c.get_or_create(1, lambda: ('w', 5)) == 'w' and 1 in c  # a later touch decodes again
