"""TensorBoard-compatible scalar sink (the scalar half of rltoolkit/tensorboard_logger.py:173-364).

The image has no tensorboard package, so events are written directly in TensorBoard's on-disk
format: a TFRecord stream of ``Event`` protobufs in ``events.out.tfevents.<time>.<host>``.
Each record is  uint64 len | uint32 masked_crc32c(len) | Event bytes | uint32 masked_crc32c(bytes);
an Event is {1: wall_time (double), 2: step (int64), 3: file_version (string) | 5: Summary}, a
Summary {1: Value*} and a Value {1: tag (string), 2: simple_value (float)}.  TensorBoard reads
these files as written; ``read_scalars`` decodes them back (tests/test_tb.py checks both CRCs).

Histograms, video and hyper-parameter panels of the reference writer are logging-only
(out of scope); the scalar tags and step axes follow the reference exactly.
"""
import os
import socket
import struct
import time

# ---------------------------------------------------------------- CRC-32C (Castagnoli), table-driven
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- minimal protobuf encoding
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _len_field(field, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _event(step, wall_time, summary=None, file_version=None) -> bytes:
    b = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        b += _len_field(3, file_version.encode())
    if summary is not None:
        b += _len_field(5, summary)
    return b


def _scalar_summary(tag, value) -> bytes:
    v = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
    return _len_field(1, v)


class ScalarWriter:
    """add_scalar(tag, value, step) into a TensorBoard event file under log_dir."""

    def __init__(self, log_dir, filename_suffix=""):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "events.out.tfevents.%d.%s%s" % (int(time.time()), socket.gethostname(),
                                                                           filename_suffix))
        self._f = open(self.path, "ab")
        self._write(_event(0, time.time(), file_version="brain.Event:2"))

    def _write(self, ev: bytes):
        if self._f is None:  # closed at the end of train(): a later log call appends to the same file
            self._f = open(self.path, "ab")
        hdr = struct.pack("<Q", len(ev))
        self._f.write(hdr + struct.pack("<I", _masked(crc32c(hdr))) + ev + struct.pack("<I", _masked(crc32c(ev))))

    def add_scalar(self, tag, value, step):
        self._write(_event(step, time.time(), summary=_scalar_summary(tag, float(value))))

    def flush(self):
        if self._f is not None:
            self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class TensorboardWriter(ScalarWriter):
    """Scalar methods of rltoolkit.tensorboard_logger.TensorboardWriter, same tags and step axes."""

    def log_running_return(self, iterations, frames, rollouts, running_return):  # :241-246
        self.add_scalar("1_Running_return/per_iterations", running_return, iterations)
        self.add_scalar("1_Running_return/per_frames", running_return, frames)
        self.add_scalar("1_Running_return/per_rollouts", running_return, rollouts)

    def log_test_return(self, iterations, frames, rollouts, test_return):  # :248-253
        self.add_scalar("1_Test_return/per_iterations", test_return, iterations)
        self.add_scalar("1_Test_return/per_frames", test_return, frames)
        self.add_scalar("1_Test_return/per_rollouts", test_return, rollouts)

    def log_loss(self, i, loss):  # :255-258
        for key, value in loss.items():
            self.add_scalar("Loss/" + key.capitalize(), value, i)

    def log_acm_pretrain_loss(self, train_loss, validation_loss, epoch):  # :260-264
        self.add_scalar("Loss/pretrain_acm_train", train_loss, epoch)
        self.add_scalar("Loss/pretrain_acm_val", validation_loss, epoch)

    def log_kl_div_updates(self, iterations, frames, rollouts, updates_no):  # :178-183
        self.add_scalar("PPO/KL_updates_mean/per_iterations", updates_no, iterations)
        self.add_scalar("PPO/KL_updates_mean/per_frames", updates_no, frames)
        self.add_scalar("PPO/KL_updates_mean/per_rollouts", updates_no, rollouts)

    def log_sac_alpha(self, iterations, alpha):  # :185-186
        self.add_scalar("SAC/Alpha_per_iterations", alpha, iterations)

    def log_action_mean_std(self, iterations, actions):  # :289-307 (actions [T, A], already denormalised)
        for j in range(actions.shape[1]):
            col = actions[:, j]
            self.add_scalar("Action/mean/%d" % j, float(col.mean()), iterations)
            self.add_scalar("Action/std/%d" % j, float(col.std()), iterations)

    def log_obs_mean_std(self, iterations, mean, std):  # :357-364
        for i in range(len(mean)):
            self.add_scalar("Obs/mean/%d" % i, float(mean[i]), iterations)
            self.add_scalar("Obs/std/%d" % i, float(std[i]), iterations)


# ---------------------------------------------------------------- reader (tests / tooling)
def _read_varint(b, i):
    v, s = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _fields(b):
    i, out = 0, []
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError("wire type %d" % w)
        out.append((f, w, v))
    return out


def read_scalars(path):
    """[(step, tag, value)] of an event file; raises on a CRC mismatch."""
    res = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if hc != _masked(crc32c(hdr)):
            raise ValueError("length crc mismatch at %d" % i)
        ev = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if dc != _masked(crc32c(ev)):
            raise ValueError("data crc mismatch at %d" % i)
        i += 16 + n
        step = 0
        for f, w, v in _fields(ev):
            if f == 2:
                step = v
            elif f == 5:
                for sf, _, val in _fields(v):
                    if sf != 1:
                        continue
                    tag, x = None, None
                    for vf, _, vv in _fields(val):
                        if vf == 1:
                            tag = vv.decode()
                        elif vf == 2:
                            (x,) = struct.unpack("<f", vv)
                    res.append((step, tag, x))
    return res
