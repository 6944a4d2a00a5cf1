"""Velodyne capture (reference include/VelodyneCapture.h:413-525) -- CPU tier.

The reference ships no capture file, so the oracle (oracle/oracle_velo.cpp) is cross-checked
against a pure-Python restatement of capturePCAP's loop on synthetic and adversarial packets, and
the pcap reader (host code of the product, bshot_pcap_load) against pcap files written here.
Parity vs the reference binary: unpinned (it cannot be built: libpcap, Boost absent)."""
import struct

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

LUT32 = bshot_py.HDL32_VERTICAL
LUT16 = [-15.0, 1.0, -13.0, 3.0, -11.0, 5.0, -9.0, 7.0, -7.0, 9.0, -5.0, 11.0, -3.0, 13.0, -1.0, 15.0]


def packets_from_rotations(frames, sensor_type=0x21):
    """HDL-32E data packets carrying synth_lasers(sensor=2) rotations: 12 firings of 32 returns per
    packet, rotational position = azimuth in 0.01 deg (a trailing partial packet is dropped)."""
    L = np.concatenate([bshot_py.synth_lasers(f, sensor=2) for f in frames])
    fir = L.reshape(-1, 32)
    npk = len(fir) // 12
    pk = np.zeros((npk, 1206), np.uint8)
    for p in range(npk):
        for f in range(12):
            F = fir[p * 12 + f]
            base = f * 100
            struct.pack_into("<HH", pk[p], base, 0xEEFF, int(round(F[0]["azimuth"] * 100)))
            for i in range(32):
                struct.pack_into("<HB", pk[p], base + 4 + 3 * i, int(F[i]["distance"]), int(F[i]["intensity"]))
        pk[p, 1204] = 0x37
        pk[p, 1205] = sensor_type
    return pk, np.arange(npk, dtype=np.int64) * 553 + 1_500_000_000_000_000


def random_packets(seed, npk, sensor_type=0x22):
    rng = np.random.default_rng(seed)
    pk = rng.integers(0, 256, (npk, 1206)).astype(np.uint8)
    for p in range(npk):
        rot = (np.arange(12) * 40 + rng.integers(0, 36000)) % 36000
        if rng.random() < 0.3:
            rot[rng.integers(0, 12)] = rng.integers(36000, 65536)  # out-of-range positions wrap once
        for f in range(12):
            struct.pack_into("<H", pk[p], f * 100 + 2, int(rot[f]))
        pk[p, 1205] = sensor_type
    return pk, rng.integers(0, 2**40, npk).astype(np.int64)


def py_decode(pk, ut, maxl, sf):
    lut = LUT16 if maxl == 16 else LUT32
    last, lasers, queue = 0.0, [], []
    for p in range(len(pk)):
        b = bytes(pk[p])
        rot = [struct.unpack_from("<H", b, f * 100 + 2)[0] for f in range(12)]
        interp = ((rot[1] + 36000) - rot[0]) / 2.0 if rot[1] < rot[0] else (rot[1] - rot[0]) / 2.0
        for f in range(12):
            for li in range(32):
                az = float(rot[f])
                if li >= maxl:
                    az += interp
                if az >= 36000:
                    az -= 36000
                if last > az:
                    sf -= 1
                if sf > 0:
                    last = az
                    continue
                if last > az:
                    queue.append(lasers)
                    lasers = []
                s = li % maxl
                d, inten = struct.unpack_from("<HB", b, f * 100 + 4 + 3 * s)
                lasers.append((az / 100.0, lut[s], d, inten, s, int(ut[p])))
                last = az
    return queue


def _cmp_oracle_py(pk, ut, maxl, sf):
    rec, cnt = orc.velodyne_decode(pk, ut, maxl, sf)
    q = py_decode(pk, ut, maxl, sf)
    assert list(cnt) == [len(r) for r in q]
    flat = [x for r in q for x in r]
    assert len(flat) == len(rec)
    for a, b in zip(rec, flat):
        assert (float(a["azimuth"]), float(a["vertical"]), int(a["distance"]), int(a["intensity"]), int(a["id"]),
                int(a["time"])) == b


@pytest.mark.parametrize("maxl,sf", [(32, 0), (32, 1), (16, 0), (16, 2), (32, -3)])
def test_oracle_matches_python_random(maxl, sf):
    pk, ut = random_packets(maxl + sf, 40)
    _cmp_oracle_py(pk, ut, maxl, sf)


def test_oracle_matches_python_synthetic_rotations():
    pk, ut = packets_from_rotations([0, 1])
    pk, ut = pk[150:260], ut[150:260]  # across the rotation split
    _cmp_oracle_py(pk, ut, 32, 0)
    rec, cnt = orc.velodyne_decode(pk, ut, 32, 0)
    assert len(cnt) == 1  # one split -> one pushed rotation, the last one is never pushed


def test_oracle_rejects_foreign_sensor_type():
    pk, ut = random_packets(3, 4, sensor_type=0x21)
    pk[2, 1205] = 0x10
    with pytest.raises(ValueError):
        orc.velodyne_decode(pk, ut)


def write_pcap(path, pk, ts, extra=True, nsec=False):
    """classic pcap: global header + records (42 B of Ethernet/IP/UDP header + 1206 B payload);
    with extra, foreign records (a 554 B position packet, a truncated capture) are interleaved."""
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B23C4D if nsec else 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i in range(len(pk)):
            sec, usec = ts[i]
            sub = usec * 1000 if nsec else usec
            data = bytes(42) + bytes(pk[i])
            f.write(struct.pack("<IIII", sec, sub, len(data), len(data)) + data)
            if extra and i % 7 == 3:
                junk = bytes(554)
                f.write(struct.pack("<IIII", sec, sub, len(junk), len(junk)) + junk)
            if extra and i % 11 == 5:
                short = bytes(100)
                f.write(struct.pack("<IIII", sec, sub, len(short), 1248) + short)


def ref_unixtime(sec, usec):
    # ss << tv_sec << std::setw(6) << std::left << std::setfill('0') << tv_usec
    return int(str(sec) + str(usec).ljust(6, "0"))


@pytest.mark.parametrize("nsec", [False, True])
def test_pcap_reader(tmp_path, nsec):
    pk, _ = random_packets(9, 30, sensor_type=0x21)
    ts = [(1_500_000_000 + i, [5, 999999, 120, 0, 34567][i % 5]) for i in range(len(pk))]
    path = tmp_path / "cap.pcap"
    write_pcap(path, pk, ts, nsec=nsec)
    got, ut = bshot_py.pcap_load(path)
    assert np.array_equal(got, pk)
    assert list(ut) == [ref_unixtime(s, u) for s, u in ts]
    assert ref_unixtime(7, 5) == 7500000  # the left-aligned fill of the reference
