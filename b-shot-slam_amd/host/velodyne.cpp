// velodyne.cpp -- PCAP file reading (host) and the velodyne::VelodyneCapture drop-in
// (include/bshot/velodyne.h) over the GPU packet decode (csrc/velodyne.hip).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/bshot/velodyne.h"

namespace {

uint32_t rd32(const unsigned char* p, bool swap) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

// capturePCAP's time stamp (include/VelodyneCapture.h:437-439):
//   ss << tv_sec << std::setw(6) << std::left << std::setfill('0') << tv_usec;  std::stoll(ss.str())
long long pcap_unixtime(uint32_t sec, uint32_t usec) {
    std::string u = std::to_string(usec);
    if (u.size() < 6) u.append(6 - u.size(), '0');
    return std::stoll(std::to_string(sec) + u);
}

}  // namespace

extern "C" int bshot_pcap_load(const char* path, uint8_t* payloads, int64_t* unixtime, int cap, int* n_packets) {
    if (!path || !n_packets || cap < 0) return BSHOT_EINVAL;
    *n_packets = 0;
    FILE* f = std::fopen(path, "rb");
    if (!f) return BSHOT_EINVAL;
    std::vector<unsigned char> buf;
    unsigned char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    std::fclose(f);
    if (buf.size() < 24) return BSHOT_EINVAL;
    const uint32_t magic = rd32(buf.data(), false);
    bool swap = false, nsec = false;
    if (magic == 0xa1b2c3d4u) {
    } else if (magic == 0xd4c3b2a1u) {
        swap = true;
    } else if (magic == 0xa1b23c4du) {
        nsec = true;
    } else if (magic == 0x4d3cb2a1u) {
        swap = nsec = true;
    } else {
        return BSHOT_EINVAL;
    }
    size_t off = 24;
    int n = 0;
    while (off + 16 <= buf.size()) {
        const uint32_t sec = rd32(&buf[off], swap), sub = rd32(&buf[off + 4], swap);
        const uint32_t incl = rd32(&buf[off + 8], swap), len = rd32(&buf[off + 12], swap);
        off += 16;
        if (off + incl > buf.size()) break;  // truncated file: pcap_next_ex reports an error
        const unsigned char* data = &buf[off];
        off += incl;
        // (:432-434) wire length - 42 != 1206 (unsigned) -> skip; a record captured shorter than the
        // packet (incl < 1248) is skipped too (the reference would read past the capture buffer)
        if (len - 42u != 1206u || incl < 1248u) continue;
        if (payloads && n < cap) {
            std::memcpy(payloads + (size_t)n * 1206, data + 42, 1206);
            unixtime[n] = pcap_unixtime(sec, nsec ? sub / 1000u : sub);
        }
        ++n;
    }
    *n_packets = n;
    return n > cap && payloads ? BSHOT_ECAP : BSHOT_OK;
}

namespace velodyne {

VelodyneCapture::VelodyneCapture() {}

VelodyneCapture::~VelodyneCapture() { close(); }

bool VelodyneCapture::open(const std::string& filename) {
    if (isRun()) close();
    int npk = 0;
    if (bshot_pcap_load(filename.c_str(), nullptr, nullptr, 0, &npk) != BSHOT_OK)
        throw std::runtime_error("VelodyneCapture: cannot read " + filename);
    std::vector<uint8_t> pk((size_t)npk * 1206);
    std::vector<int64_t> ut((size_t)npk);
    if (npk > 0 && bshot_pcap_load(filename.c_str(), pk.data(), ut.data(), npk, &npk) != BSHOT_OK)
        throw std::runtime_error("VelodyneCapture: cannot read " + filename);
    bshot_ctx* c = nullptr;
    if (bshot_create(&c, device_, nullptr) != BSHOT_OK) throw std::runtime_error("VelodyneCapture: bshot_create");
    std::vector<Laser> all((size_t)npk * 384);
    std::vector<int32_t> rs((size_t)npk * 384 + 2), rc((size_t)npk * 384 + 2);
    int nrot = 0, nout = 0;
    const int rc0 = bshot_velodyne_decode(c, pk.data(), ut.data(), npk, MAX_NUM_LASERS, specifiedframe,
                                          reinterpret_cast<bshot_laser*>(all.data()), (int)all.size(), rs.data(),
                                          rc.data(), (int)rs.size(), &nrot, &nout);
    const std::string err = rc0 ? bshot_last_error(c) : "";
    bshot_destroy(c);
    if (rc0 != BSHOT_OK) throw std::runtime_error("VelodyneCapture: " + err);
    for (int i = 0; i < nrot; ++i) queue_.emplace_back(all.begin() + rs[i], all.begin() + rs[i] + rc[i]);
    filename_ = filename;
    opened_ = true;
    return true;
}

bool VelodyneCapture::isOpen() { return opened_; }

bool VelodyneCapture::isRun() { return !queue_.empty(); }

void VelodyneCapture::close() {
    opened_ = false;
    filename_.clear();
    std::deque<std::vector<Laser>>().swap(queue_);
}

void VelodyneCapture::retrieve(std::vector<Laser>& lasers, const bool sort) {
    if (queue_.empty()) return;
    lasers = queue_.front();
    if (sort) std::sort(lasers.begin(), lasers.end());
    queue_.pop_front();
}

}  // namespace velodyne
