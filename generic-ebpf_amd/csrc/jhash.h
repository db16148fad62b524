// jhash.h — the hashtable maps' key hash: Bob Jenkins' lookup3 "hashlittle" (public domain,
// 2006), which is what the reference's ebpf_jenkins_hash() is on little-endian hosts
// (sys/dev/ebpf/ebpf_jhash.h:159-330 via Linux/ebpf/user/ebpf_linux_user.c:204-208).
// The reference reads the key in 4-, 2- or 1-byte pieces depending on its alignment; all three
// paths compute the same value, so this restatement reads bytes.  Pinned by
// tests/golden/maps/jhash.npz (generated from the reference header, tools/gen_golden_jhash.py).
// Plain C++ usable from host code and HIP device code.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define EBPF_JHASH_FN __host__ __device__ inline
#else
#define EBPF_JHASH_FN inline
#endif

EBPF_JHASH_FN uint32_t
ebpf_jhash_rot(uint32_t x, int k)
{
	return (x << k) | (x >> (32 - k));
}

EBPF_JHASH_FN uint32_t
ebpf_jhash(const void *key, size_t length, uint32_t initval)
{
	const uint8_t *k = static_cast<const uint8_t *>(key);
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + (uint32_t)length + initval;
	auto word = [](const uint8_t *p) {
		return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
	};
	while (length > 12) {
		a += word(k);
		b += word(k + 4);
		c += word(k + 8);
		// mix(a, b, c)
		a -= c; a ^= ebpf_jhash_rot(c, 4);  c += b;
		b -= a; b ^= ebpf_jhash_rot(a, 6);  a += c;
		c -= b; c ^= ebpf_jhash_rot(b, 8);  b += a;
		a -= c; a ^= ebpf_jhash_rot(c, 16); c += b;
		b -= a; b ^= ebpf_jhash_rot(a, 19); a += c;
		c -= b; c ^= ebpf_jhash_rot(b, 4);  b += a;
		length -= 12;
		k += 12;
	}
	if (length == 0)
		return c;
	// the last 1..12 bytes, zero-padded, into (a, b, c)
	uint8_t t[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
	for (size_t i = 0; i < length; i++)
		t[i] = k[i];
	a += word(t);
	b += word(t + 4);
	c += word(t + 8);
	// final(a, b, c)
	c ^= b; c -= ebpf_jhash_rot(b, 14);
	a ^= c; a -= ebpf_jhash_rot(c, 11);
	b ^= a; b -= ebpf_jhash_rot(a, 25);
	c ^= b; c -= ebpf_jhash_rot(b, 16);
	a ^= c; a -= ebpf_jhash_rot(c, 4);
	b ^= a; b -= ebpf_jhash_rot(a, 14);
	c ^= b; c -= ebpf_jhash_rot(b, 24);
	return c;
}
