"""Dependency-free TensorBoard scalar writer + the per-rank logger.

Reference: ``PerRankLogger`` (`labs/tiny/train_tiny.py:34-67`)
prints ``[rank r | step N] k=v ...``, appends it to ``out/log.rank{r}.txt``
and writes scalars with ``torch.utils.tensorboard`` to ``out/tb/rank{r}``.
The ``tensorboard`` package is not installed in this image, so the event
file is produced directly: TFRecord framing (length, masked CRC-32C, payload,
masked CRC-32C) around hand-encoded ``Event{wall_time, step, summary{value{tag,
simple_value}}}`` protobufs — readable by any TensorBoard.
"""
import os
import socket
import struct
import time

_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c):
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _len_field(tag, payload):
    return bytes([tag]) + _varint(len(payload)) + payload


def encode_event(wall_time, step=None, file_version=None, scalars=None):
    ev = b"\x09" + struct.pack("<d", wall_time)
    if step is not None:
        ev += b"\x10" + _varint(int(step))
    if file_version is not None:
        ev += _len_field(0x1A, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = _len_field(0x0A, tag.encode()) + b"\x15" + struct.pack("<f", float(v))
            summ += _len_field(0x0A, val)
        ev += _len_field(0x2A, summ)
    return ev


def frame(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", _masked(crc32c(hdr))) + payload + struct.pack("<I", _masked(crc32c(payload)))


def read_events(path):
    """Decode our own event files back to [(step, {tag: value})] (tests)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        payload = data[i + 12:i + 12 + n]
        assert struct.unpack_from("<I", data, i + 12 + n)[0] == _masked(crc32c(payload))
        i += 16 + n
        step, scalars, j = None, {}, 9
        while j < len(payload):
            tag = payload[j]
            j += 1
            if tag == 0x10:
                step, j = _read_varint(payload, j)
            elif tag in (0x1A, 0x2A):
                ln, j = _read_varint(payload, j)
                if tag == 0x2A:
                    scalars.update(_parse_summary(payload[j:j + ln]))
                j += ln
        if scalars:
            out.append((step, scalars))
    return out


def _read_varint(b, j):
    n = s = 0
    while True:
        x = b[j]
        j += 1
        n |= (x & 0x7F) << s
        s += 7
        if not x & 0x80:
            return n, j


def _parse_summary(b):
    res, j = {}, 0
    while j < len(b):
        j += 1
        ln, j = _read_varint(b, j)
        v = b[j:j + ln]
        j += ln
        k = 1
        tl, k = _read_varint(v, k)
        tag = v[k:k + tl].decode()
        k += tl
        res[tag] = struct.unpack_from("<f", v, k + 1)[0]
    return res


class SummaryWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self._f = open(self.path, "ab")
        self._f.write(frame(encode_event(time.time(), file_version="brain.Event:2")))

    def add_scalar(self, tag, value, step):
        self._f.write(frame(encode_event(time.time(), step=step, scalars={tag: value})))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


class PerRankLogger:
    """``[rank r | step N] k=v ...`` to stdout + ``log.rank{r}.txt`` + ``tb/rank{r}`` scalars."""

    def __init__(self, out_dir, rank, use_tb=True):
        os.makedirs(out_dir, exist_ok=True)
        self.rank = rank
        self.fh = open(os.path.join(out_dir, f"log.rank{rank}.txt"), "a", buffering=1)
        self.tb = SummaryWriter(os.path.join(out_dir, "tb", f"rank{rank}")) if use_tb else None

    def log(self, step, logs: dict):
        line = f"[rank {self.rank} | step {step}] " + " ".join(f"{k}={v}" for k, v in logs.items())
        print(line, flush=True)
        self.fh.write(line + "\n")
        if self.tb:
            for k, v in logs.items():
                if isinstance(v, (int, float)):
                    self.tb.add_scalar(k, v, step)

    def close(self):
        self.fh.close()
        if self.tb:
            self.tb.flush()
            self.tb.close()
