/* TEST INFRASTRUCTURE ONLY (container): golden vectors for the reference's key hash.
 * Compiles the reference's own sys/dev/ebpf/ebpf_jhash.h (included from where it lies under
 * /root/reference, never copied) and prints jenkins_hash() of keys read from stdin, so that
 * tests/golden/jhash.npz pins the engine's restatement (csrc/jhash.h) and the oracle's.
 * Input lines: "<initval> <offset> <hex key>" (offset 0..3 places the key at that misalignment,
 * exercising the header's aligned / half-aligned / byte paths).  Output: one hash per line. */
#include <endian.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifndef BYTE_ORDER
#define BYTE_ORDER __BYTE_ORDER
#endif
#ifndef LITTLE_ENDIAN
#define LITTLE_ENDIAN __LITTLE_ENDIAN
#endif
#include "dev/ebpf/ebpf_jhash.h"

int
main(void)
{
	static char line[4096];
	static uint8_t buf[2048] __attribute__((aligned(16)));
	while (fgets(line, sizeof(line), stdin)) {
		unsigned long initval, off;
		char hex[2048] = "";
		if (sscanf(line, "%lu %lu %2047s", &initval, &off, hex) < 2)
			continue;
		if (strcmp(hex, "-") == 0)
			hex[0] = 0;
		size_t n = strlen(hex) / 2;
		for (size_t i = 0; i < n; i++) {
			unsigned v;
			sscanf(hex + 2 * i, "%2x", &v);
			buf[off + i] = (uint8_t)v;
		}
		printf("%u\n", jenkins_hash(buf + off, n, (uint32_t)initval));
	}
	return 0;
}
