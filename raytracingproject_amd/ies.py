"""IES photometric files for the IES Texture node (host side).

A restatement of util/util_ies.cpp (IESFile::parse / process / pack) and of
LightManager::device_update_ies (render/light.cpp:1080-1125), which lays the
slots out in the `__ies` array the kernel reads (kernel/svm/svm_ies.h): an
offset table with one entry per slot (-1 for an invalid file), then per valid
slot h_num, v_num (as int bits), the horizontal and vertical angles in radians
and the h_num x v_num candela table converted to Watt/sr.
"""
from __future__ import annotations

import re

import numpy as np

_F = np.float32
_DOUBLE = re.compile(rb"[ \t\n\v\f\r]*([+-]?(?:\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?))")
_LONG = re.compile(rb"[ \t\n\v\f\r]*([+-]?\d+)")


class _TextParser:
    """IESTextParser (util_ies.cpp:76-119): commas are blanks, reading starts
    at "\\nTILT=", strtod / strtol semantics (a failed read ends the input)."""

    def __init__(self, text: bytes):
        self.text = text.replace(b",", b" ")
        i = self.text.find(b"\nTILT=")
        self.pos = None if i < 0 else i

    def eof(self) -> bool:
        return self.pos is None or self.pos >= len(self.text) or self.text[self.pos] == 0

    def _get(self, pattern, conv):
        if self.eof():
            return conv(b"0")
        m = pattern.match(self.text, self.pos)
        if not m:
            self.pos = None
            return conv(b"0")
        self.pos = m.end()
        return conv(m.group(1))

    def get_double(self) -> float:
        return self._get(_DOUBLE, float)

    def get_long(self) -> int:
        return self._get(_LONG, int)


class IESFile:
    """util_ies.h IESFile: h_angles, v_angles (float32, degrees until
    processed, then radians) and intensity[h][v] (float32)."""

    TYPE_B, TYPE_C = 2, 1

    def __init__(self, content: str | bytes):
        self.h_angles: list = []
        self.v_angles: list = []
        self.intensity: list = []
        data = content.encode() if isinstance(content, str) else bytes(content)
        self.content = data
        if not (self._parse(data) and self._process()):
            self.h_angles, self.v_angles, self.intensity = [], [], []

    # util_ies.cpp:121-208
    def _parse(self, ies: bytes) -> bool:
        if not ies:
            return False
        p = _TextParser(ies)
        if p.eof():
            return False
        if p.text.startswith(b"\nTILT=INCLUDE", p.pos):
            p.pos += 13
            p.get_double()
            num_tilt = p.get_long()
            for _ in range(2 * num_tilt):
                p.get_double()
        else:
            i = p.text.find(b"\n", p.pos + 1)
            p.pos = None if i < 0 else i
        if p.eof():
            return False
        p.pos += 1
        p.get_long()
        p.get_double()
        factor = p.get_double()
        v_num = p.get_long()
        h_num = p.get_long()
        self.type = p.get_long()
        if self.type not in (self.TYPE_B, self.TYPE_C):
            return False
        p.get_long()
        p.get_double()
        p.get_double()
        p.get_double()
        factor *= p.get_double()
        factor *= p.get_double()
        p.get_double()
        factor *= 0.0706650768394  # candela -> Watt/sr (4 pi / 177.83)
        self.v_angles = [_F(p.get_double()) for _ in range(v_num)]
        self.h_angles = [_F(p.get_double()) for _ in range(h_num)]
        self.intensity = [[_F(factor * p.get_double()) for _ in range(v_num)] for _ in range(h_num)]
        return not p.eof()

    # util_ies.cpp:210-296
    def _process_type_b(self) -> bool:
        self.intensity = [[self.intensity[j][i] for j in range(len(self.h_angles))] for i in range(len(self.v_angles))]
        self.h_angles, self.v_angles = self.v_angles, self.h_angles
        h = self.h_angles
        if h[-1] != _F(90.0):
            return False
        if h[0] == _F(0.0):
            hnum = len(h)
            nh = [_F(_F(90.0) - h[i]) for i in range(hnum - 1, 0, -1)] + [_F(_F(90.0) + h[i]) for i in range(hnum)]
            ni = [self.intensity[i] for i in range(hnum - 1, 0, -1)] + [self.intensity[i] for i in range(hnum)]
            self.h_angles, self.intensity = nh, ni
        elif h[0] == _F(-90.0):
            self.h_angles = [_F(a + _F(90.0)) for a in h]
        self.h_angles.append(_F(360.0))
        self.intensity.append(self.intensity[0])
        v = self.v_angles
        if v[-1] != _F(90.0):
            return False
        if v[0] == _F(0.0):
            vnum = len(v)
            self.v_angles = [_F(_F(90.0) - v[i]) for i in range(vnum - 1, 0, -1)] + \
                            [_F(_F(90.0) + v[i]) for i in range(vnum)]
            self.intensity = [[row[j] for j in range(vnum - 2, -1, -1)] + list(row) for row in self.intensity]
        elif v[0] == _F(-90.0):
            self.v_angles = [_F(a + _F(90.0)) for a in v]
        return True

    # util_ies.cpp:298-371
    def _process_type_c(self) -> bool:
        h = self.h_angles
        if h[0] == _F(90.0):
            h = self.h_angles = [_F(a - _F(90.0)) for a in h]
        if h[0] != _F(0.0):
            return False
        if len(h) == 1:
            h.append(_F(360.0))
            self.intensity.append(self.intensity[0])
        if h[-1] == _F(90.0):
            hnum = len(h)
            for i in range(hnum - 2, -1, -1):
                h.append(_F(_F(180.0) - h[i]))
                self.intensity.append(self.intensity[i])
        if h[-1] == _F(180.0):
            hnum = len(h)
            for i in range(hnum - 2, -1, -1):
                h.append(_F(_F(360.0) - h[i]))
                self.intensity.append(self.intensity[i])
        if h[-1] != _F(360.0):
            hnum = len(h)
            last_step = _F(h[hnum - 1] - h[hnum - 2])
            first_step = _F(h[1] - h[0])
            difference = _F(_F(360.0) - h[hnum - 1])
            if last_step == difference or first_step == difference:
                h.append(_F(360.0))
                self.intensity.append(self.intensity[0])
            else:
                return False
        v_first, v_last = self.v_angles[0], self.v_angles[-1]
        if v_first == _F(90.0):
            if v_last == _F(180.0):
                self.v_angles = [_F(_F(180.0) - a) for a in self.v_angles]
            else:
                return False
        elif v_first != _F(0.0):
            return False
        return True

    # util_ies.cpp:373-404
    def _process(self) -> bool:
        if not self.h_angles or not self.v_angles:
            return False
        if not (self._process_type_b() if self.type == self.TYPE_B else self._process_type_c()):
            return False
        k = _F(_F(np.pi) / _F(180.0))  # M_PI_F / 180.f
        self.v_angles = [_F(a * k) for a in self.v_angles]
        self.h_angles = [_F(a * k) for a in self.h_angles]
        return True

    def packed_size(self) -> int:
        if self.v_angles and self.h_angles:
            return 2 + len(self.h_angles) + len(self.v_angles) + len(self.h_angles) * len(self.v_angles)
        return 0

    def pack(self) -> np.ndarray:
        """util_ies.cpp:58-74"""
        if not self.packed_size():
            return np.zeros(0, np.float32)
        head = np.array([len(self.h_angles), len(self.v_angles)], dtype=np.int32).view(np.float32)
        body = [np.asarray(self.h_angles, np.float32), np.asarray(self.v_angles, np.float32)]
        body += [np.asarray(row, np.float32) for row in self.intensity]
        return np.concatenate([head] + body).astype(np.float32)


def pack_slots(slots: list[IESFile]) -> np.ndarray:
    """LightManager::device_update_ies: the offset table, then the packed slots."""
    offset = len(slots)
    table = np.zeros(len(slots), np.float32)
    parts = []
    for i, f in enumerate(slots):
        size = f.packed_size()
        if size > 0:
            table[i] = np.int32(offset).view(np.float32)
            parts.append(f.pack())
            offset += size
        else:
            table[i] = np.int32(-1).view(np.float32)
    return np.concatenate([table] + parts).astype(np.float32)
