"""Retry policies (reference core/common/src/main/java/alluxio/retry/*.java).

``RetryPolicy.attempt()`` returns True while another attempt is allowed, sleeping between
attempts as the policy dictates — the same shape as the reference's ``RetryPolicy`` so that
client code reads ``while policy.attempt(): try ...``.
"""
from __future__ import annotations

import random
import time


class RetryPolicy:
    def __init__(self):
        self._attempt_count = 0

    @property
    def attempt_count(self) -> int:
        return self._attempt_count

    def attempt(self) -> bool:
        if self._attempt_count == 0:
            self._attempt_count = 1
            return True
        if not self._may_continue():
            return False
        delay = self._sleep_time()
        if delay > 0:
            time.sleep(delay)
        self._attempt_count += 1
        return True

    def _may_continue(self) -> bool:
        raise NotImplementedError

    def _sleep_time(self) -> float:
        return 0.0


class CountingRetry(RetryPolicy):
    def __init__(self, max_retries: int):
        super().__init__()
        self.max_retries = max_retries

    def _may_continue(self) -> bool:
        return self._attempt_count <= self.max_retries


class ExponentialBackoffRetry(RetryPolicy):
    def __init__(self, base_sleep_ms: int, max_sleep_ms: int, max_retries: int):
        super().__init__()
        self.base = base_sleep_ms
        self.max = max_sleep_ms
        self.max_retries = max_retries

    def _may_continue(self) -> bool:
        return self._attempt_count <= self.max_retries

    def _sleep_time(self) -> float:
        ms = min(self.max, self.base * (1 << min(self._attempt_count - 1, 30)))
        return ms * (1.0 + random.random() * 0.1) / 1000.0


class TimeoutRetry(RetryPolicy):
    def __init__(self, timeout_ms: int, sleep_ms: int):
        super().__init__()
        self.deadline = time.monotonic() + timeout_ms / 1000.0
        self.sleep_ms = sleep_ms

    def _may_continue(self) -> bool:
        return time.monotonic() < self.deadline

    def _sleep_time(self) -> float:
        return self.sleep_ms / 1000.0


class ExponentialTimeBoundedRetry(RetryPolicy):
    def __init__(self, max_duration_ms: int, initial_sleep_ms: int, max_sleep_ms: int):
        super().__init__()
        self.deadline = time.monotonic() + max_duration_ms / 1000.0
        self.next_sleep = initial_sleep_ms
        self.max_sleep = max_sleep_ms

    def _may_continue(self) -> bool:
        return time.monotonic() < self.deadline

    def _sleep_time(self) -> float:
        s = min(self.next_sleep, max(0.0, (self.deadline - time.monotonic()) * 1000.0))
        self.next_sleep = min(self.max_sleep, self.next_sleep * 2)
        return s / 1000.0


def retry(fn, policy: RetryPolicy, retry_on=(Exception,)):
    last = None
    while policy.attempt():
        try:
            return fn()
        except retry_on as e:  # noqa: PERF203
            last = e
    if last is not None:
        raise last
    raise RuntimeError("retry policy allowed no attempts")
