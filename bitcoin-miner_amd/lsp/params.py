"""LSP parameters -- mirror of src/github.com/cmu440/lsp/params.go:8-35."""
from __future__ import annotations

from dataclasses import dataclass

DefaultEpochLimit = 5
DefaultEpochMillis = 2000
DefaultWindowSize = 1


@dataclass
class Params:
    EpochLimit: int = DefaultEpochLimit    # epochs of silence before a connection is lost (K)
    EpochMillis: int = DefaultEpochMillis  # epoch duration (delta)
    WindowSize: int = DefaultWindowSize    # max unacknowledged data messages in flight (omega)
    # Not in params.go: times each originated datagram is sent (lsp/endpoint.py); 1 is the
    # protocol exactly as specified, and what every lsp test runs.
    SendCopies: int = 1

    def __str__(self) -> str:
        return f"[EpochLimit: {self.EpochLimit}, EpochMillis: {self.EpochMillis}, WindowSize: {self.WindowSize}]"


def NewParams() -> Params:
    return Params()
