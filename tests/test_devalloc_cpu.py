"""devalloc.configure_device_allocator: the trainer loop's allocator settings (no device here)."""

import torch

from pipelinerl_amd import devalloc


def _fake_device(monkeypatch):
    applied = []
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(devalloc, "_set_allocator_settings", applied.append)
    for k in devalloc.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    return applied


def test_default_rounds_request_sizes(monkeypatch):
    applied = _fake_device(monkeypatch)
    monkeypatch.setattr(devalloc, "_applied", None)
    assert devalloc.configure_device_allocator() == devalloc.DEFAULT_SETTINGS
    assert applied == [devalloc.DEFAULT_SETTINGS]
    assert devalloc.rounding_allowance() == 1.25  # the coarsest interval: 4 divisions


def test_user_environment_wins(monkeypatch):
    applied = _fake_device(monkeypatch)
    monkeypatch.setenv("PYTORCH_HIP_ALLOC_CONF", "garbage_collection_threshold:0.8")
    assert devalloc.configure_device_allocator() is None and applied == []


def test_disabled_or_no_device(monkeypatch):
    applied = _fake_device(monkeypatch)
    assert devalloc.configure_device_allocator("") is None
    assert devalloc.configure_device_allocator(None) is None
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    assert devalloc.configure_device_allocator() is None
    assert applied == []


def test_division_counts_and_allowance(monkeypatch):
    assert devalloc.divisions("roundup_power2_divisions:[512:16,>:4]") == [16, 4]
    assert devalloc.divisions("garbage_collection_threshold:0.8,roundup_power2_divisions:8") == [8]
    assert devalloc.divisions("max_split_size_mb:512") == []
    monkeypatch.setattr(devalloc, "_applied", None)
    for k in devalloc.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    assert devalloc.rounding_allowance() == 1.0
    monkeypatch.setenv("PYTORCH_HIP_ALLOC_CONF", "roundup_power2_divisions:8")
    assert devalloc.rounding_allowance() == 1.125
    monkeypatch.setenv("PYTORCH_HIP_ALLOC_CONF", "roundup_power2_divisions:1")
    assert devalloc.rounding_allowance() == 1.0
