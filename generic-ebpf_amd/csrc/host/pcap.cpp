// pcap.cpp — a packet capture as a batch (the path starts in host memory,
// "a NIC ring or pcap buffer").  The classic libpcap file format: a 24-byte global header
// (magic, version, thiszone, sigfigs, snaplen, linktype) and per packet a 16-byte record header
// (ts_sec, ts_usec or ts_nsec, incl_len, orig_len) followed by incl_len captured bytes.  The
// magic tells the byte order and the timestamp unit: 0xa1b2c3d4 (microseconds) or 0xa1b23c4d
// (nanoseconds), as written or byte-swapped.
//
// The records' captured bytes are gathered into one buffer in offsets form (ebpf_pkt_batch:
// packet i = data[offsets[i], offsets[i+1])), which ebpf_prog_run_batch consumes directly; the
// program sees each packet's captured bytes, as a caller that hands a record's buffer to the
// reference's ebpf_prog_run would.  ebpf_pcap_extents skips the gather: the batch is the capture
// itself in extents form (each record's (start, end) in the capture; the 16-byte record headers
// stay between the packets and are never part of one).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.h"

namespace {

// buffers this file handed out: pinned (hipHostMalloc) or not (malloc)
std::mutex g_lock;
std::unordered_map<const void *, bool> g_bufs;

uint32_t
rd32(const uint8_t *p, bool swap)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return swap ? __builtin_bswap32(v) : v;
}

void *
alloc(size_t bytes, bool pinned)
{
	if (bytes == 0)
		bytes = 1;
	if (pinned) {
		int n = 0;
		void *p = nullptr;
		if (hipGetDeviceCount(&n) == hipSuccess && n > 0 &&
		    hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) {
			std::lock_guard<std::mutex> g(g_lock);
			g_bufs[p] = true;
			return p;
		}
		(void)hipGetLastError(); // no GPU: pageable memory instead
	}
	void *p = malloc(bytes);
	if (p) {
		std::lock_guard<std::mutex> g(g_lock);
		g_bufs[p] = false;
	}
	return p;
}

void
release(const void *p)
{
	if (!p)
		return;
	bool pinned;
	{
		std::lock_guard<std::mutex> g(g_lock);
		auto it = g_bufs.find(p);
		if (it == g_bufs.end())
			return; // not ours
		pinned = it->second;
		g_bufs.erase(it);
	}
	if (pinned)
		(void)hipHostFree(const_cast<void *>(p));
	else
		free(const_cast<void *>(p));
}

// The capture's global header and a validating walk over its record headers.
struct pcap_scan {
	bool swap = false, nsec = false;
	uint32_t snaplen = 0, linktype = 0;
	uint64_t count = 0, bytes = 0, truncated = 0, cut = 0;
};

int
scan_capture(const void *capture, size_t len, pcap_scan *sc)
{
	if (!capture || len < 24) {
		set_last_error("pcap: NULL argument or shorter than the 24-byte global header");
		return EINVAL;
	}
	const uint8_t *b = static_cast<const uint8_t *>(capture);
	uint32_t magic;
	memcpy(&magic, b, 4);
	switch (magic) {
	case 0xa1b2c3d4u: sc->swap = false; sc->nsec = false; break;
	case 0xa1b23c4du: sc->swap = false; sc->nsec = true; break;
	case 0xd4c3b2a1u: sc->swap = true; sc->nsec = false; break;
	case 0x4d3cb2a1u: sc->swap = true; sc->nsec = true; break;
	default:
		set_last_error("pcap: unknown magic (not a classic libpcap capture)");
		return EINVAL;
	}
	const bool swap = sc->swap;
	sc->snaplen = rd32(b + 16, swap);
	sc->linktype = rd32(b + 20, swap);
	const uint32_t snaplen = sc->snaplen;
	// count the records and their bytes, validating every header
	size_t at = 24;
	while (at < len) {
		if (len - at < 16) {
			set_last_error("pcap: truncated record header at byte " + std::to_string(at));
			return EINVAL;
		}
		const uint32_t incl = rd32(b + at + 8, swap), orig = rd32(b + at + 12, swap);
		if (incl > len - at - 16) {
			set_last_error("pcap: record at byte " + std::to_string(at) + " runs past the end");
			return EINVAL;
		}
		// a record longer than the header's snaplen (some writers get the snaplen wrong): as
		// libpcap's reader does, the packet is its first snaplen bytes (counted as truncated)
		const uint32_t keep = (snaplen && incl > snaplen) ? snaplen : incl;
		sc->cut += keep < incl;
		sc->truncated += keep < orig;
		sc->count++;
		sc->bytes += keep;
		at += 16 + (size_t)incl;
	}
	return 0;
}

void
fill_info(const pcap_scan &sc, struct ebpf_pcap_info *info)
{
	if (!info)
		return;
	info->linktype = sc.linktype;
	info->snaplen = sc.snaplen;
	info->nanosecond = sc.nsec ? 1u : 0u;
	info->byte_swapped = sc.swap ? 1u : 0u;
	info->truncated = sc.truncated;
	info->bytes = sc.bytes;
}

} // namespace

EBPF_EXPORT int
ebpf_pcap_batch(const void *capture, size_t len, int pinned, struct ebpf_pkt_batch *batch,
		struct ebpf_pcap_info *info)
{
	pcap_scan sc;
	if (!batch) {
		set_last_error("pcap: NULL batch");
		return EINVAL;
	}
	if (int err = scan_capture(capture, len, &sc))
		return err;
	const uint8_t *b = static_cast<const uint8_t *>(capture);
	const bool swap = sc.swap;
	const uint32_t snaplen = sc.snaplen;
	const uint64_t count = sc.count, bytes = sc.bytes, cut = sc.cut;
	size_t at;
	// pass 2: gather the captured bytes
	uint8_t *data = static_cast<uint8_t *>(alloc((size_t)bytes, pinned != 0));
	uint64_t *offs = static_cast<uint64_t *>(alloc((size_t)(count + 1) * sizeof(uint64_t), pinned != 0));
	if (!data || !offs) {
		release(data);
		release(offs);
		return ENOMEM;
	}
	// where record i's bytes start in the capture: 24 + 16 (i + 1) + offs[i] unless a record
	// was cut to the snaplen (then from a table)
	std::vector<size_t> src;
	if (cut) {
		try {
			src.resize(count);
		} catch (...) {
			release(data);
			release(offs);
			return ENOMEM;
		}
	}
	uint64_t o = 0, i = 0;
	at = 24;
	while (at < len) {
		const uint32_t incl = rd32(b + at + 8, swap);
		if (cut)
			src[i] = at + 16;
		offs[i++] = o;
		o += (snaplen && incl > snaplen) ? snaplen : incl;
		at += 16 + (size_t)incl;
	}
	offs[count] = o;
	// the copies are independent, so large captures are gathered by several threads (contiguous
	// packet ranges)
	auto gather = [&](uint64_t lo, uint64_t hi) {
		for (uint64_t k = lo; k < hi; k++)
			memcpy(data + offs[k], b + (cut ? src[k] : 24 + 16 * (k + 1) + offs[k]),
			       (size_t)(offs[k + 1] - offs[k]));
	};
	unsigned nt = std::thread::hardware_concurrency();
	nt = std::max(1u, std::min(nt, 16u));
	if (bytes < (16u << 20) || count < 4096)
		nt = 1;
	if (nt == 1) {
		gather(0, count);
	} else {
		std::vector<std::thread> th;
		unsigned t = 0;
		try {
			for (; t < nt; t++)
				th.emplace_back(gather, count * t / nt, count * (t + 1) / nt);
		} catch (...) { // no thread to be had: this one copies the ranges not started
			gather(count * t / nt, count);
		}
		for (std::thread &x : th)
			x.join();
	}
	memset(batch, 0, sizeof(*batch));
	batch->data = data;
	batch->offsets = offs;
	batch->count = count;
	fill_info(sc, info);
	return 0;
}

EBPF_EXPORT int
ebpf_pcap_extents(const void *capture, size_t len, int pinned, struct ebpf_pkt_batch *batch,
		  struct ebpf_pcap_info *info)
{
	pcap_scan sc;
	if (!batch) {
		set_last_error("pcap: NULL batch");
		return EINVAL;
	}
	if (int err = scan_capture(capture, len, &sc))
		return err;
	const uint8_t *b = static_cast<const uint8_t *>(capture);
	uint64_t *ext = static_cast<uint64_t *>(alloc((size_t)sc.count * 2 * sizeof(uint64_t), pinned != 0));
	if (!ext)
		return ENOMEM;
	// record i's captured bytes in place: (start, start + kept length)
	uint64_t i = 0;
	for (size_t at = 24; at < len; i++) {
		const uint32_t incl = rd32(b + at + 8, sc.swap);
		const uint32_t keep = (sc.snaplen && incl > sc.snaplen) ? sc.snaplen : incl;
		ext[2 * i] = at + 16;
		ext[2 * i + 1] = at + 16 + keep;
		at += 16 + (size_t)incl;
	}
	memset(batch, 0, sizeof(*batch));
	batch->data = capture;
	batch->offsets = ext;
	batch->count = sc.count;
	batch->flags = EBPF_BATCH_EXTENTS;
	fill_info(sc, info);
	return 0;
}

EBPF_EXPORT void
ebpf_pcap_batch_free(struct ebpf_pkt_batch *batch)
{
	if (!batch)
		return;
	release(batch->data); // (an extents batch's data is the caller's capture: not ours, kept)
	release(batch->offsets);
	batch->data = nullptr;
	batch->offsets = nullptr;
	batch->count = 0;
	batch->flags = 0;
}
