/*
 * ebpf_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference interpreter.
 *
 * Follows generic-ebpf sys/dev/ebpf/ebpf_interpreter.c:23-372 case by case (line numbers in
 * the comments), compiled for x86-64 exactly as the reference is: shift counts are masked to
 * 5/6 bits (x86 SHL/SHR semantics, SURVEY.md Appendix A [probed]).  It agrees with the golden
 * vectors under tests/golden/; run-result parity is unpinned (see ebpf_oracle.h).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this file.
 */
#include "ebpf_oracle.h"

#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

enum {
	F_NONE = 0, F_BAD_OPCODE = 1, F_DIV_ZERO = 2, F_MEM = 3, F_SLOT = 4, F_HELPER = 5,
	F_HELPER_UNSUPPORTED = 6, F_BAD_REG = 7, F_LOOP = 8, F_MAP_WRITE = 9, F_BAD_MAP = 10,
	F_WRITES = 11,
	F_UNDEF = 100 /* oracle only (oracle_prog.track_undef): a read of a stack byte no store wrote */
};

#define STACK_BYTES 512

struct region_env {
	uint64_t pkt_lo, pkt_hi;
	uint64_t stk_lo, stk_hi;
	const struct oracle_prog *p;
	uint8_t *sdef; /* track_undef: 1 per stack byte a store wrote (NULL: not tracked) */
	int map_hit;   /* check_access: the map whose values hold the access, else -1 */
};

/* 0 = ok, else a fault code. write=1 for stores (into map values too: ebpf_interpreter.c:343-366
 * writes through whatever pointer the program holds; re->map_hit tells the caller). */
static inline int
check_access(struct region_env *re, uint64_t addr, uint64_t size, int write)
{
	re->map_hit = -1;
	uint64_t end = addr + size;
	if (end < addr)
		return F_MEM;
	if (addr >= re->pkt_lo && end <= re->pkt_hi)
		return 0;
	if (addr >= re->stk_lo && end <= re->stk_hi) {
		if (re->sdef) {
			uint8_t *d = re->sdef + (addr - re->stk_lo);
			for (uint64_t i = 0; i < size; i++)
				if (!write && !d[i]) /* (stores mark their bytes in taint_pre) */
					return F_UNDEF;
		}
		return 0;
	}
	for (uint32_t m = 0; m < re->p->nmaps; m++) {
		const struct oracle_map *mp = &re->p->maps[m];
		uint64_t lo = (uint64_t)(uintptr_t)mp->data;
		uint64_t hi = lo + (uint64_t)mp->value_size * mp->max_entries;
		if (!(addr >= lo && end <= hi))
			continue;
		/* a hashtable value is its own allocation (a hash_elem, ebpf_map_hashtable.c:30-36):
		 * an access that leaves it reads stray memory, which stops the packet like any other */
		if (mp->kind == ORACLE_MAP_HASH && (addr - lo) / mp->value_size != (end - 1 - lo) / mp->value_size)
			continue;
		re->map_hit = (int)m;
		return 0;
	}
	return F_MEM;
}

static inline uint64_t
load_n(uint64_t addr, int size)
{
	const void *ptr = (const void *)(uintptr_t)addr;
	switch (size) {
	case 1: { uint8_t v; memcpy(&v, ptr, 1); return v; }
	case 2: { uint16_t v; memcpy(&v, ptr, 2); return v; }
	case 4: { uint32_t v; memcpy(&v, ptr, 4); return v; }
	default: { uint64_t v; memcpy(&v, ptr, 8); return v; }
	}
}

static inline void
store_n(uint64_t addr, int size, uint64_t v)
{
	void *ptr = (void *)(uintptr_t)addr;
	switch (size) {
	case 1: { uint8_t x = (uint8_t)v; memcpy(ptr, &x, 1); break; }
	case 2: { uint16_t x = (uint16_t)v; memcpy(ptr, &x, 2); break; }
	case 4: { uint32_t x = (uint32_t)v; memcpy(ptr, &x, 4); break; }
	default: memcpy(ptr, &v, 8); break;
	}
}

static inline uint16_t bs16(uint16_t x) { return (uint16_t)((x >> 8) | (x << 8)); }

/* The 90 opcodes with a case in ebpf_interpreter.c:41-366. */
static const uint8_t k_valid_ops[] = {
	0x04, 0x0c, 0x14, 0x1c, 0x24, 0x2c, 0x34, 0x3c, 0x44, 0x4c, 0x54, 0x5c, 0x64, 0x6c,
	0x74, 0x7c, 0x84, 0x94, 0x9c, 0xa4, 0xac, 0xb4, 0xbc, 0xc4, 0xcc, 0xd4, 0xdc,
	0x07, 0x0f, 0x17, 0x1f, 0x27, 0x2f, 0x37, 0x3f, 0x47, 0x4f, 0x57, 0x5f, 0x67, 0x6f,
	0x77, 0x7f, 0x87, 0x97, 0x9f, 0xa7, 0xaf, 0xb7, 0xbf, 0xc7, 0xcf,
	0x61, 0x69, 0x71, 0x79, 0x62, 0x6a, 0x72, 0x7a, 0x63, 0x6b, 0x73, 0x7b, 0x18,
	0x05, 0x15, 0x1d, 0x25, 0x2d, 0x35, 0x3d, 0x45, 0x4d, 0x55, 0x5d, 0x65, 0x6d, 0x75,
	0x7d, 0x85, 0x95, 0xa5, 0xad, 0xb5, 0xbd, 0xc5, 0xcd, 0xd5, 0xdd,
};

static uint8_t k_valid_tab[256];

__attribute__((constructor)) static void
init_valid_tab(void)
{
	for (unsigned i = 0; i < sizeof(k_valid_ops); i++)
		k_valid_tab[k_valid_ops[i]] = 1;
}

static inline int
valid_op(uint8_t op)
{
	return k_valid_tab[op];
}

/* Which opcodes name a dst / src register (reg[inst->dst] / reg[inst->src] in the reference). */
static inline int
uses_dst(uint8_t op)
{
	return !(op == 0x05 || op == 0x85 || op == 0x95);
}

static inline int
uses_src(uint8_t op)
{
	uint8_t cls = op & 7;
	if (cls == 1 || cls == 3) /* LDX, STX */
		return 1;
	if ((cls == 4 || cls == 7 || cls == 5) && (op & 0x08)) {
		/* REG-source ALU/JMP; LE/BE (0xd4/0xdc) and CALL/EXIT never read src */
		if (op == 0xdc || op == 0x8d || op == 0x9d || op == 0x85 || op == 0x95)
			return 0;
		return 1;
	}
	return 0;
}

static inline uint32_t
rot32(uint32_t x, int k)
{
	return (x << k) | (x >> (32 - k));
}

uint32_t
oracle_jhash(const void *key, uint32_t length, uint32_t initval)
{
	const uint8_t *k = (const uint8_t *)key;
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + length + initval;
#define W(p) ((uint32_t)(p)[0] | (uint32_t)(p)[1] << 8 | (uint32_t)(p)[2] << 16 | (uint32_t)(p)[3] << 24)
	while (length > 12) {
		a += W(k);
		b += W(k + 4);
		c += W(k + 8);
		a -= c; a ^= rot32(c, 4);  c += b;
		b -= a; b ^= rot32(a, 6);  a += c;
		c -= b; c ^= rot32(b, 8);  b += a;
		a -= c; a ^= rot32(c, 16); c += b;
		b -= a; b ^= rot32(a, 19); a += c;
		c -= b; c ^= rot32(b, 4);  b += a;
		length -= 12;
		k += 12;
	}
	if (length == 0)
		return c;
	uint8_t t[12] = {0};
	memcpy(t, k, length);
	a += W(t);
	b += W(t + 4);
	c += W(t + 8);
#undef W
	c ^= b; c -= rot32(b, 14);
	a ^= c; a -= rot32(c, 11);
	b ^= a; b -= rot32(a, 25);
	c ^= b; c -= rot32(b, 16);
	a ^= c; a -= rot32(c, 4);
	b ^= a; b -= rot32(a, 14);
	c ^= b; c -= rot32(b, 24);
	return c;
}

void
oracle_hash_build(struct oracle_map *m)
{
	for (uint32_t b = 0; b < m->nbuckets; b++)
		m->bucket_head[b] = -1;
	for (uint32_t i = 0; i < m->max_entries; i++) {
		uint32_t b = oracle_jhash(m->keys + (uint64_t)m->key_size * i, m->key_size, 0) &
			     (m->nbuckets - 1);
		m->bucket_next[i] = m->bucket_head[b];
		m->bucket_head[b] = (int32_t)i;
	}
}

/* ebpf_map_lookup_elem (ebpf_map.c:77-84) → array_map_lookup_elem (ebpf_map_array.c:115-124)
 * or hashtable_map_lookup_elem (ebpf_map_hashtable.c:285-301) */
static inline uint64_t
helper_map_lookup(struct region_env *re, int checked, uint64_t r1, uint64_t r2, int *fault)
{
	const struct oracle_prog *p = re->p;
	if (r1 == 0 || r2 == 0) /* em == NULL || key == NULL → NULL (ebpf_map.c:80-81) */
		return 0;
	const struct oracle_map *m = NULL;
	for (uint32_t i = 0; i < p->nmaps; i++)
		if (p->maps[i].handle == r1) {
			m = &p->maps[i];
			break;
		}
	if (m == NULL) {
		*fault = F_BAD_MAP;
		return 0;
	}
	if (m->kind == ORACLE_MAP_HASH) {
		/* hashtable_map_lookup_elem (ebpf_map_hashtable.c:285-301): the element whose key
		 * equals the key_size bytes at r2 (how the reference finds it — bucket, chain — does
		 * not change which value that is) */
		if (checked) {
			int f = check_access(re, r2, m->key_size, 0);
			if (f) {
				*fault = f;
				return 0;
			}
		}
		const void *key = (const void *)(uintptr_t)r2;
		if (m->nbuckets) {
			uint32_t b = oracle_jhash(key, m->key_size, 0) & (m->nbuckets - 1);
			for (int32_t i = m->bucket_head[b]; i >= 0; i = m->bucket_next[i])
				if (memcmp(m->keys + (uint64_t)m->key_size * i, key, m->key_size) == 0)
					return (uint64_t)(uintptr_t)(m->data + (uint64_t)m->value_size * i);
			return 0;
		}
		for (uint32_t i = 0; i < m->max_entries; i++)
			if (memcmp(m->keys + (uint64_t)m->key_size * i, key, m->key_size) == 0)
				return (uint64_t)(uintptr_t)(m->data + (uint64_t)m->value_size * i);
		return 0;
	}
	if (checked) {
		int f = check_access(re, r2, 4, 0);
		if (f) {
			*fault = f;
			return 0;
		}
	}
	uint32_t k = (uint32_t)load_n(r2, 4);
	if (k >= m->max_entries)
		return 0;
	return (uint64_t)(uintptr_t)(m->data + (uint64_t)m->value_size * k);
}

/* ---- map-writing helpers, device-batch semantics (ebpf_oracle.h) ---- */
enum { WR_HELPER = 0, WR_STORE = 1, WR_ADD = 2 };
struct wrec {
	uint64_t pkt;
	uint32_t seq;
	uint32_t map;
	uint32_t key;  /* array: the key; hashtable: op (1 update, 2 delete) | flags << 8;
			* WR_STORE / WR_ADD into a hashtable: the element's index */
	uint64_t voff; /* value bytes in the log's arena (hashtable: key_size bytes, then the value) */
	uint8_t kind;  /* WR_HELPER: update / delete; WR_STORE / WR_ADD: a store into a value */
	uint8_t size;  /* WR_STORE / WR_ADD: bytes */
	uint32_t off;  /* ... byte offset in the map's values (hashtable: in the element's value) */
	uint64_t data; /* ... the stored bytes (WR_ADD: the addend), little-endian */
};
struct wlog {
	struct wrec *rec;
	size_t n, cap;
	uint8_t *arena;
	size_t used, arena_cap;
};
static __thread struct wlog *t_wlog; /* set by oracle_run_batch per thread */
static __thread uint64_t t_pkt;
static __thread uint32_t t_seq;
static __thread uint32_t t_writes; /* the packet's logged writes (ebpf_oracle.h: at most 16) */
static __thread int t_sequential; /* oracle_prog.sequential: writes land at once */
static __thread int t_loops;      /* the batch's program loops (prog_has_loops) */
static __thread int t_rb;         /* ... and reads its counter updates back (prog_reads_counters) */
#define ORACLE_WRITES_MAX 16u /* include/ebpf_gpu.h EBPF_FAULT_WRITES (dprog.h DP_WRITES_MAX) */
#define ORACLE_OVL_WORDS 32u  /* the packet's own view: 8-byte words of map values (DP_OVL_MAX) */
static __thread struct {
	uint32_t n;
	uint64_t w[ORACLE_OVL_WORDS]; /* map index << 56 | element << 16 | word within the value(s) */
} t_words;

/* A program with loops that reads its counter updates back keeps the packet's view of the map
 * values it changed in 32 words (ebpf_oracle.h): the store or counter update of `size` bytes at
 * byte `voff` of element `elem`'s value (arrays: elem 0 and voff from the first value — their
 * values are contiguous; hashtables: each value starts on 8 bytes, as the device's slots place
 * them) takes the 8-byte words it touches that the packet has not yet touched; F_WRITES when
 * they do not fit (before anything happens), else 0. */
static int
take_words(int mi, uint64_t elem, uint64_t voff, int size)
{
	uint64_t need[2];
	uint32_t k = 0;
	for (uint64_t w = voff >> 3; w <= (voff + (uint64_t)size - 1) >> 3; w++) {
		const uint64_t key = (uint64_t)mi << 56 | elem << 16 | w;
		uint32_t i = 0;
		while (i < t_words.n && t_words.w[i] != key)
			i++;
		if (i == t_words.n)
			need[k++] = key;
	}
	if (t_words.n + k > ORACLE_OVL_WORDS)
		return F_WRITES;
	for (uint32_t i = 0; i < k; i++)
		t_words.w[t_words.n++] = need[i];
	return 0;
}

/* A logged write of the batch (a map_update_elem / map_delete_elem that succeeds, a store into a
 * map value other than an aligned counter update into an array, any counter update into a
 * hashtable's value): 0, or F_WRITES for the packet's 17th.  Only in
 * batch mode, and only for a program with loops: a loop-free program writes as often as its path
 * says, like the reference (ebpf_interpreter.c:343-366, ebpf_map.c:101-108 ->
 * ebpf_map_array.c:198-211 run every store and update they reach); the reference's own run,
 * sequential or one packet, has no limit at all. */
static inline int
count_write(void)
{
	if (t_sequential || t_wlog == NULL || !t_loops)
		return 0;
	return ++t_writes > ORACLE_WRITES_MAX ? F_WRITES : 0;
}

static void
wlog_push2(uint32_t map, uint32_t key, const uint8_t *a, uint32_t na, const uint8_t *b, uint32_t nb)
{
	struct wlog *w = t_wlog;
	if (w == NULL)
		return; /* single-packet oracle_run: the write is not kept */
	if (w->n == w->cap) {
		w->cap = w->cap ? 2 * w->cap : 1024;
		w->rec = realloc(w->rec, w->cap * sizeof(*w->rec));
	}
	if (w->used + na + nb > w->arena_cap) {
		w->arena_cap = (w->arena_cap ? 2 * w->arena_cap : 65536) + na + nb;
		w->arena = realloc(w->arena, w->arena_cap);
	}
	memcpy(w->arena + w->used, a, na);
	if (nb)
		memcpy(w->arena + w->used + na, b, nb);
	w->rec[w->n++] = (struct wrec){t_pkt, t_seq++, map, key, w->used, WR_HELPER, 0, 0, 0};
	w->used += na + nb;
}

/* ---- stores into map values, batch semantics (ebpf_oracle.h) ----
 * The packet's own stores: one entry per byte it stored into a map value (addresses in the
 * oracle's map storage), newest last.  Its loads read them back; the maps stay the batch-start
 * bytes until the batch's records are applied. */
#define OVL_MAX 8192
struct ovl {
	uint32_t n;
	uint64_t addr[OVL_MAX];
	uint8_t byte[OVL_MAX];
};
static __thread struct ovl *t_ovl; /* batch mode (not sequential): the packet's overlay */

static int
ovl_find(uint64_t a)
{
	for (uint32_t i = t_ovl->n; i-- > 0;)
		if (t_ovl->addr[i] == a)
			return (int)i;
	return -1;
}

/* 0, or F_MEM when the packet stored more bytes than the overlay holds (never in the tests;
 * the device bounds its overlay by the program's stores per path) */
static int
ovl_put(uint64_t a, uint8_t b)
{
	int k = ovl_find(a);
	if (k < 0) {
		if (t_ovl->n == OVL_MAX)
			return F_MEM;
		k = (int)t_ovl->n++;
		t_ovl->addr[k] = a;
	}
	t_ovl->byte[k] = b;
	return 0;
}

/* A load of map-value bytes: the packet's own stores over the batch-start bytes. */
static inline uint64_t
load_mem(uint64_t addr, int size)
{
	if (t_ovl == NULL || t_ovl->n == 0)
		return load_n(addr, size);
	uint64_t v = 0;
	for (int i = 0; i < size; i++) {
		const int k = ovl_find(addr + (uint64_t)i);
		const uint8_t b = k >= 0 ? t_ovl->byte[k] : *(const uint8_t *)(uintptr_t)(addr + (uint64_t)i);
		v |= (uint64_t)b << (8 * i);
	}
	return v;
}

/* A store of `size` bytes of v at addr inside the values of map mi (check_access): in place when
 * the run is sequential (or a lone oracle_run), else into the packet's overlay and the batch's
 * log.  `add`: a counter update adding `delta` (the caller checked the alignment).  Returns 0 or
 * a fault code. */
static int
value_store(const struct region_env *re, int mi, uint64_t addr, int size, uint64_t v, int add,
	    uint64_t delta)
{
	const struct oracle_map *m = &re->p->maps[mi];
	struct wlog *w = t_wlog;
	if (t_sequential || w == NULL || t_ovl == NULL) {
		store_n(addr, size, v);
		return 0;
	}
	if (!add || m->kind == ORACLE_MAP_HASH) { /* (a hashtable's counter updates are records) */
		int f = count_write();
		if (f)
			return f;
	}
	if (t_loops && t_rb) {
		const uint64_t o = addr - (uint64_t)(uintptr_t)m->data;
		int f = m->kind == ORACLE_MAP_HASH ? take_words(mi, o / m->value_size, o % m->value_size, size)
						   : take_words(mi, 0, o, size);
		if (f)
			return f;
	}
	for (int i = 0; i < size; i++) {
		int f = ovl_put(addr + (uint64_t)i, (uint8_t)(v >> (8 * i)));
		if (f)
			return f;
	}
	uint64_t off = addr - (uint64_t)(uintptr_t)m->data;
	uint32_t elem = 0;
	if (m->kind == ORACLE_MAP_HASH) {
		elem = (uint32_t)(off / m->value_size);
		off %= m->value_size;
	}
	if (w->n == w->cap) {
		w->cap = w->cap ? 2 * w->cap : 1024;
		w->rec = realloc(w->rec, w->cap * sizeof(*w->rec));
	}
	const uint64_t mask = size == 8 ? ~0ull : (1ull << (8 * size)) - 1;
	w->rec[w->n++] = (struct wrec){t_pkt, t_seq++, (uint32_t)mi, elem, 0, add ? WR_ADD : WR_STORE,
				       (uint8_t)size, (uint32_t)off, (add ? delta : v) & mask};
	return 0;
}

/* Is a counter update at addr (map mi) aligned to its width within the map's values? */
static inline int
value_aligned(const struct region_env *re, int mi, uint64_t addr, int size)
{
	const struct oracle_map *m = &re->p->maps[mi];
	uint64_t off = addr - (uint64_t)(uintptr_t)m->data;
	if (m->kind == ORACLE_MAP_HASH)
		off %= m->value_size;
	return off % (uint64_t)size == 0;
}

/* Counter-update tracking (ebpf_oracle.h): LDX{W,DW} X = [P + off]; ADD/SUB X; STX [P + off] = X,
 * consecutive (JA aside).  cnt_next() is called with every executed instruction before it runs;
 * it returns 1 when this instruction is the pattern's store. */
struct cnt_track {
	int stage; /* 0 none, 1 after the load, 2 after the add */
	uint8_t x, p;
	int16_t off;
	int size;
	uint64_t loaded;
};

static inline int
cnt_next(struct cnt_track *ct, uint8_t op, uint8_t d, uint8_t s, int16_t off, int std)
{
	if (op == 0x05)
		return 0; /* JA: not a step (the device folds it into the state graph) */
	if (ct->stage == 1 && d == ct->x) {
		int ok = 0;
		switch (op) {
		case 0x07: case 0x17: ok = 1; break;                    /* ADD64 / SUB64 imm */
		case 0x0f: case 0x1f: ok = s != ct->x; break;           /* ... reg */
		case 0xb7: ok = !std; break;                            /* reference MOV64 = add */
		case 0xbf: ok = !std && s != ct->x; break;
		case 0x04: case 0x14: ok = ct->size == 4; break;        /* ALU32 ADD / SUB imm */
		case 0x0c: case 0x1c: ok = ct->size == 4 && s != ct->x; break;
		}
		ct->stage = ok ? 2 : 0;
		return 0;
	}
	if (ct->stage == 2) {
		ct->stage = 0;
		const uint8_t stx = ct->size == 8 ? 0x7b : 0x63;
		return op == stx && d == ct->p && s == ct->x && off == ct->off;
	}
	ct->stage = 0;
	return 0;
}

/* after an LDX of `size` bytes into d from [s + off] that loaded v */
static inline void
cnt_load(struct cnt_track *ct, uint8_t d, uint8_t s, int16_t off, int size, uint64_t v)
{
	if ((size == 4 || size == 8) && d != s)
		*ct = (struct cnt_track){1, d, s, off, size, v};
}

/* STX / ST / XADD of `size` bytes of v at a (already region-checked, re->map_hit set) */
static inline int
mem_store(const struct region_env *re, int checked, uint64_t a, int size, uint64_t v, int add,
	  uint64_t delta)
{
	if (checked && re->map_hit >= 0) {
		if (add && !value_aligned(re, re->map_hit, a, size))
			add = 0;
		return value_store(re, re->map_hit, a, size, v, add, delta);
	}
	store_n(a, size, v);
	return 0;
}

static void
wlog_push(uint32_t map, uint32_t key, const uint8_t *value, uint32_t vs)
{
	wlog_push2(map, key, value, vs, NULL, 0);
}

static const struct oracle_map *
find_map(const struct oracle_prog *p, uint64_t handle, uint32_t *idx)
{
	for (uint32_t i = 0; i < p->nmaps; i++)
		if (p->maps[i].handle == handle) {
			*idx = i;
			return &p->maps[i];
		}
	return NULL;
}

/* ebpf_map_update_elem (ebpf_map.c:101-108) -> array_map_update_elem (ebpf_map_array.c:185-211) */
static inline uint64_t
helper_map_update(struct region_env *re, int checked, uint64_t r1, uint64_t r2, uint64_t r3,
		  uint64_t r4, int *fault)
{
	if (r1 == 0 || r2 == 0 || r3 == 0 || r4 > 2) /* EBPF_EXIST = 2 */
		return 22;                             /* EINVAL */
	uint32_t mi;
	const struct oracle_map *m = find_map(re->p, r1, &mi);
	if (m == NULL) {
		*fault = F_BAD_MAP;
		return 0;
	}
	if (m->kind == ORACLE_MAP_HASH) {
		/* hashtable_map_update_elem (ebpf_map_hashtable.c:346-390) against the batch-start
		 * table: check_update_flags (:87-100) by the key's presence, EBUSY for a new key when
		 * the table is full (:371-377); the value is read only by a call that succeeds */
		if (checked && (*fault = check_access(re, r2, m->key_size, 0)))
			return 0;
		const int exists = helper_map_lookup(re, 0, r1, r2, fault) != 0;
		const uint32_t cap = m->capacity ? m->capacity : m->max_entries;
		uint64_t rc = exists && (r4 & 1) ? 17 : !exists && (r4 & 2) ? 2
			      : !exists && m->max_entries >= cap ? 16 : 0;
		if (rc == 0) {
			if (checked && (*fault = check_access(re, r3, m->value_size, 0)))
				return 0;
			if ((*fault = count_write()))
				return 0;
			wlog_push2(mi, 1u | (uint32_t)r4 << 8, (const uint8_t *)(uintptr_t)r2, m->key_size,
				   (const uint8_t *)(uintptr_t)r3, m->value_size);
		}
		return rc;
	}
	if (r4 & 1)  /* EBPF_NOEXIST: every key of an array exists */
		return 17; /* EEXIST */
	if (checked && (*fault = check_access(re, r2, 4, 0)))
		return 0;
	const uint32_t k = (uint32_t)load_n(r2, 4);
	if (k >= m->max_entries)
		return 22;
	if (checked && (*fault = check_access(re, r3, m->value_size, 0)))
		return 0;
	if (t_sequential) { /* the reference: memcpy into the value now (ebpf_map_array.c:173-183) */
		memmove(m->data + (uint64_t)m->value_size * k, (const void *)(uintptr_t)r3, m->value_size);
		return 0;
	}
	if ((*fault = count_write()))
		return 0;
	wlog_push(mi, k, (const uint8_t *)(uintptr_t)r3, m->value_size);
	return 0;
}

/* ebpf_map_delete_elem (ebpf_map.c) -> array_map_delete_elem (ebpf_map_array.c:246-250) */
static inline uint64_t
helper_map_delete(struct region_env *re, int checked, uint64_t r1, uint64_t r2, int *fault)
{
	uint32_t mi;
	if (r1 == 0 || r2 == 0) /* ebpf_map.c:130-136: checked before the map is touched */
		return 22;        /* EINVAL */
	const struct oracle_map *m = find_map(re->p, r1, &mi);
	if (m == NULL) {
		*fault = F_BAD_MAP;
		return 0;
	}
	if (m->kind == ORACLE_MAP_HASH) {
		/* hashtable_map_delete_elem (ebpf_map_hashtable.c:475-502): 0 whatever the table
		 * holds; the key is hashed (read) first */
		if (checked && (*fault = check_access(re, r2, m->key_size, 0)))
			return 0;
		if ((*fault = count_write()))
			return 0;
		wlog_push2(mi, 2u, (const uint8_t *)(uintptr_t)r2, m->key_size, NULL, 0);
		return 0;
	}
	return 22; /* EINVAL: an array map (no delete) */
}

/* CALL :282-284 — helper id imm of the configured table */
static inline uint64_t
helper_call(struct region_env *re, int checked, int32_t imm, const uint64_t *reg, int *fault)
{
	const struct oracle_prog *p = re->p;
	if (imm < 0 || imm >= 64 || p->helper_kind[imm] == ORACLE_HELPER_UNSET) {
		*fault = F_HELPER;
		return 0;
	}
	switch (p->helper_kind[imm]) {
	case ORACLE_HELPER_MAP_LOOKUP:
		return helper_map_lookup(re, checked, reg[1], reg[2], fault);
	case ORACLE_HELPER_MAP_UPDATE:
		return helper_map_update(re, checked, reg[1], reg[2], reg[3], reg[4], fault);
	case ORACLE_HELPER_MAP_DELETE:
		return helper_map_delete(re, checked, reg[1], reg[2], fault);
	default:
		*fault = F_HELPER_UNSUPPORTED;
		return 0;
	}
}


/* track_undef (test tooling): taint[r] = r holds a value derived from an address (r1, r10, a
 * map handle, a lookup result), whose bits differ between the reference, this oracle and the
 * device; a result, a packet byte, a branch or a map key that depends on one is undefined.
 * The stack shadow sdef holds 2 for a byte of a stored tainted value.  Returns F_UNDEF or 0;
 * called before the instruction executes (CALL results are tainted after it). */
static int
taint_pre(const struct region_env *re, uint8_t *taint, uint8_t op, int d, int s, int16_t off,
	  int32_t imm, const uint64_t *reg, int std)
{
	const struct oracle_prog *p = re->p;
	const int cls = op & 7;
	if (d >= 11 || s >= 11)
		return 0;
	if (cls == 4 || cls == 7) { /* ALU32 / ALU64 */
		const int x = op & 0x08, code = op & 0xf0;
		if (code == 0xb0 && cls == 4) /* MOV32 */
			taint[d] = x ? taint[s] : 0;
		else if (std && code == 0xb0) /* standard MOV64 moves (the reference's adds) */
			taint[d] = x ? taint[s] : 0;
		else if (std && code == 0x80) /* standard NEG / NEG64: -dst */
			;
		else if (code == 0x80 && cls == 4) /* NEG32 = -imm */
			taint[d] = 0;
		else if (code == 0xd0) /* LE / BE: the source bit picks the order, no register is read */
			;
		else if (x && code == 0x10 && taint[d] && taint[s]) /* pointer - pointer */
			taint[d] = 0;
		else if (x)
			taint[d] |= taint[s];
		return 0;
	}
	if (op == 0x18)
		return 0; /* (taint_lddw after it executes: a map handle is an address) */
	if (cls == 5) { /* JMP */
		if (op == 0x05 || op == 0x95 || op == 0x85) {
			if (op == 0x95 && taint[0])
				return F_UNDEF;
			if (op == 0x85 && imm >= 0 && imm < 64 && re->sdef) {
				const int k = p->helper_kind[imm];
				uint32_t ks = 4, vs = 0;
				for (uint32_t m = 0; m < p->nmaps; m++)
					if (p->maps[m].handle == reg[1]) {
						if (p->maps[m].kind == ORACLE_MAP_HASH)
							ks = p->maps[m].key_size;
						vs = p->maps[m].value_size;
					}
				uint64_t rg[2] = {reg[2], reg[3]};
				uint32_t sz[2] = {ks, k == ORACLE_HELPER_MAP_UPDATE ? vs : 0};
				for (int q = 0; q < 2; q++)
					for (uint32_t i = 0; i < sz[q]; i++) {
						uint64_t a = rg[q] + i;
						if (a >= re->stk_lo && a < re->stk_hi && re->sdef[a - re->stk_lo] == 2)
							return F_UNDEF;
					}
			}
			return 0;
		}
		const int x = op & 0x08;
		if (taint[d] && !(x == 0 && imm == 0 && ((op & 0xf0) == 0x10 || (op & 0xf0) == 0x50)))
			return F_UNDEF; /* (a NULL test of a lookup result is defined) */
		if (x && taint[s])
			return F_UNDEF;
		return 0;
	}
	if (cls == 1) { /* LDX: a tainted stack byte taints the loaded value */
		const int sz = (op & 0x18) == 0x10 ? 1 : (op & 0x18) == 0x08 ? 2 : (op & 0x18) == 0 ? 4 : 8;
		uint64_t a = reg[s] + (uint64_t)(int64_t)off;
		uint8_t t = 0;
		if (re->sdef && a >= re->stk_lo && a + sz >= a && a + sz <= re->stk_hi)
			for (int i = 0; i < sz; i++)
				t |= re->sdef[a - re->stk_lo + i] == 2;
		taint[d] = t;
		return 0;
	}
	if (cls == 3 || cls == 2) { /* STX / ST */
		const int sz = (op & 0x18) == 0x10 ? 1 : (op & 0x18) == 0x08 ? 2 : (op & 0x18) == 0 ? 4 : 8;
		const uint8_t t = cls == 3 ? taint[s] : 0;
		uint64_t a = reg[d] + (uint64_t)(int64_t)off;
		if (re->sdef && a >= re->stk_lo && a + sz >= a && a + sz <= re->stk_hi) {
			for (int i = 0; i < sz; i++)
				re->sdef[a - re->stk_lo + i] = t ? 2 : 1;
			return 0;
		}
		return t ? F_UNDEF : 0;
	}
	return 0;
}

static inline uint64_t
run_ref(const struct oracle_prog *p, int checked, uint8_t *pkt, uint64_t len, uint8_t *fault_out,
	uint64_t *steps_out)
{
	uint64_t reg[11];
	uint8_t stack[STACK_BYTES], sdef[STACK_BYTES];
	struct region_env re;
	uint64_t idx = 0; /* slot index; the reference keeps a pointer (inst) */
	uint32_t pc = 0;  /* u32 as in ebpf_interpreter.c:26 */
	uint64_t steps = 0;
	int fault = F_NONE;
	uint64_t r0 = 0;

	if (checked) /* raw mode leaves the stack undefined, exactly like the reference */
		memset(stack, p->stack_init, sizeof(stack));
	for (int i = 0; i < 11; i++)
		reg[i] = p->reg_init;
	reg[1] = (uint64_t)(uintptr_t)pkt;                   /* :35 */
	reg[10] = (uint64_t)(uintptr_t)(stack + STACK_BYTES); /* :36 */
	re.pkt_lo = (uint64_t)(uintptr_t)pkt;
	re.pkt_hi = re.pkt_lo + len;
	re.stk_lo = (uint64_t)(uintptr_t)stack;
	re.stk_hi = re.stk_lo + STACK_BYTES;
	re.sdef = p->track_undef ? sdef : NULL;
	if (re.sdef)
		memset(sdef, 0, sizeof(sdef));
	uint8_t taint[11] = {0};
	taint[1] = taint[10] = 1;
	re.p = p;
	re.map_hit = -1;
	struct cnt_track ct = {0, 0, 0, 0, 0, 0};

	for (;;) {
		/* :39  inst = inst + pc++;  (cumulative stepping) */
		uint64_t cur_idx = idx + (uint64_t)pc;
		uint32_t cur_pc = pc + 1;
		idx = cur_idx;
		pc = cur_pc;
		if (idx >= p->nslots) {
			fault = F_SLOT;
			break;
		}
		const uint8_t *ip = p->insns + idx * 8;
		uint8_t op = ip[0];
		uint8_t d = ip[1] & 0x0f, s = ip[1] >> 4;
		int16_t off;
		int32_t imm;
		memcpy(&off, ip + 2, 2);
		memcpy(&imm, ip + 4, 4);
		steps++;
		if (!valid_op(op)) {
			fault = F_BAD_OPCODE; /* :367-369 */
			break;
		}
		if ((uses_dst(op) && d >= 11) || (uses_src(op) && s >= 11)) {
			fault = F_BAD_REG;
			break;
		}
		uint64_t D = d < 11 ? reg[d] : 0, S = s < 11 ? reg[s] : 0;
		uint32_t D32 = (uint32_t)D, S32 = (uint32_t)S, I32 = (uint32_t)imm;
		uint64_t IS = (uint64_t)(int64_t)imm; /* int32 imm promoted to u64 (sign-extended) */
		int taken = -1;                        /* -1: not a conditional jump */
		int msize = 0;

		if (re.sdef && (fault = taint_pre(&re, taint, op, d, s, off, imm, reg, 0)))
			break;
		const int cnt = cnt_next(&ct, op, d, s, off, 0);
		switch (op) {
		/* ---- ALU32 :41-133 — operands truncated to u32, result zero-extended ---- */
		case 0x0c: reg[d] = (uint32_t)(D32 + S32); break;
		case 0x04: reg[d] = (uint32_t)(D32 + I32); break;
		case 0x1c: reg[d] = (uint32_t)(D32 - S32); break;
		case 0x14: reg[d] = (uint32_t)(D32 - I32); break;
		case 0x2c: reg[d] = (uint32_t)(D32 * S32); break;
		case 0x24: reg[d] = (uint32_t)(D32 * I32); break;
		case 0x3c: if (!S32) { fault = F_DIV_ZERO; break; } reg[d] = D32 / S32; break;
		case 0x34: if (!I32) { fault = F_DIV_ZERO; break; } reg[d] = D32 / I32; break;
		case 0x4c: reg[d] = D32 | S32; break;
		case 0x44: reg[d] = D32 | I32; break;
		case 0x5c: reg[d] = D32 & S32; break;
		case 0x54: reg[d] = D32 & I32; break;
		case 0x6c: reg[d] = (uint32_t)(D32 << (S32 & 31)); break;
		case 0x64: reg[d] = (uint32_t)(D32 << (I32 & 31)); break;
		case 0x7c: reg[d] = D32 >> (S32 & 31); break;
		case 0x74: reg[d] = D32 >> (I32 & 31); break;
		case 0x84: reg[d] = (uint32_t)(0u - I32); break;          /* :89-91 NEG ignores dst */
		case 0x9c: if (!S32) { fault = F_DIV_ZERO; break; } reg[d] = D32 % S32; break;
		case 0x94: if (!I32) { fault = F_DIV_ZERO; break; } reg[d] = D32 % I32; break;
		case 0xac: reg[d] = D32 ^ S32; break;
		case 0xa4: reg[d] = D32 ^ I32; break;
		case 0xbc: reg[d] = S32; break;                            /* :104-106 */
		case 0xb4: reg[d] = I32; break;                            /* :107-109 */
		case 0xcc: reg[d] = D32 >> (S32 & 31); break;              /* :110-112 logical */
		case 0xc4: reg[d] = D32 >> (I32 & 31); break;              /* :113-115 logical */
		case 0xd4:                                                 /* :116-124 LE (x86: identity) */
			if (imm == 16) reg[d] = (uint16_t)D;
			else if (imm == 32) reg[d] = D32;
			break;
		case 0xdc:                                                 /* :125-133 BE = bswap on x86 */
			if (imm == 16) reg[d] = bs16((uint16_t)D);
			else if (imm == 32) reg[d] = __builtin_bswap32(D32);
			else if (imm == 64) reg[d] = __builtin_bswap64(D);
			break;
		/* ---- ALU64 :134-208 ---- */
		case 0x0f: reg[d] = D + S; break;
		case 0x07: reg[d] = D + IS; break;
		case 0x1f: reg[d] = D - S; break;
		case 0x17: reg[d] = D - IS; break;
		case 0x2f: reg[d] = D * S; break;
		case 0x27: reg[d] = D * IS; break;
		case 0x3f: if (!S) { fault = F_DIV_ZERO; break; } reg[d] = D / S; break;
		case 0x37: if (!IS) { fault = F_DIV_ZERO; break; } reg[d] = D / IS; break;
		case 0x4f: reg[d] = D | S; break;
		case 0x47: reg[d] = D | IS; break;
		case 0x5f: reg[d] = D & S; break;
		case 0x57: reg[d] = D & IS; break;
		case 0x6f: reg[d] = D << (S & 63); break;
		case 0x67: reg[d] = D << (IS & 63); break;
		case 0x7f: reg[d] = D >> (S & 63); break;
		case 0x77: reg[d] = D >> (IS & 63); break;
		case 0x87: reg[d] = D - IS; break;                          /* :182-184 NEG64 = dst - imm */
		case 0x9f: if (!S) { fault = F_DIV_ZERO; break; } reg[d] = D % S; break;
		case 0x97: if (!IS) { fault = F_DIV_ZERO; break; } reg[d] = D % IS; break;
		case 0xaf: reg[d] = D ^ S; break;
		case 0xa7: reg[d] = D ^ IS; break;
		case 0xbf: reg[d] = D + S; break;                           /* :197-199 MOV64 adds */
		case 0xb7: reg[d] = D + IS; break;                          /* :200-202 */
		case 0xcf: reg[d] = D >> (S & 63); break;                   /* :203-205 logical */
		case 0xc7: reg[d] = D >> (IS & 63); break;                  /* :206-208 logical */
		/* ---- JMP :209-326 ---- */
		case 0x05: taken = 1; break;
		case 0x1d: taken = D == S; break;
		case 0x15: taken = D == IS; break;
		case 0x2d: taken = D > S; break;
		case 0x25: taken = D > IS; break;
		case 0x3d: taken = D >= S; break;
		case 0x35: taken = D >= IS; break;
		case 0x4d: taken = (D & S) != 0; break;
		case 0x45: taken = (D & IS) != 0; break;
		case 0x5d: taken = D != S; break;
		case 0x55: taken = D != IS; break;
		case 0x6d: taken = (int64_t)D > (int64_t)S; break;
		case 0x65: taken = (int64_t)D > (int64_t)IS; break;
		case 0x7d: taken = (int64_t)D >= (int64_t)S; break;
		case 0x75: taken = (int64_t)D >= (int64_t)IS; break;
		case 0xad: taken = D < S; break;
		case 0xa5: taken = D < IS; break;
		case 0xbd: taken = D <= S; break;
		case 0xb5: taken = D <= IS; break;
		case 0xcd: taken = (int64_t)D < (int64_t)S; break;
		case 0xc5: taken = (int64_t)D < (int64_t)IS; break;
		case 0xdd: taken = (int64_t)D <= (int64_t)S; break;
		case 0xd5: taken = (int64_t)D <= (int64_t)IS; break;
		case 0x85: {                                                /* :282-284 CALL */
			uint64_t r = helper_call(&re, checked, imm, reg, &fault);
			if (!fault)
				reg[0] = r;
			break;
		}
		case 0x95: r0 = reg[0]; goto done;                          /* :285-286 EXIT */
		/* ---- memory :327-366 ---- */
		case 0x71: msize = 1; goto ldx;
		case 0x69: msize = 2; goto ldx;
		case 0x61: msize = 4; goto ldx;
		case 0x79: msize = 8;
		ldx: {
			uint64_t a = S + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 0)))
				break;
			reg[d] = checked && re.map_hit >= 0 ? load_mem(a, msize) : load_n(a, msize);
			cnt_load(&ct, d, s, off, msize, reg[d]);
			break;
		}
		case 0x18:                                                  /* :339-342 LDDW */
			if (idx + 1 >= p->nslots) { fault = F_SLOT; break; }
			{
				int32_t hi;
				memcpy(&hi, p->insns + (idx + 1) * 8 + 4, 4);
				reg[d] = (uint64_t)I32 | ((uint64_t)(uint32_t)hi << 32);
			}
			pc++;
			break;
		case 0x73: msize = 1; goto stx;
		case 0x6b: msize = 2; goto stx;
		case 0x63: msize = 4; goto stx;
		case 0x7b: msize = 8;
		stx: {
			uint64_t a = D + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 1)))
				break;
			fault = mem_store(&re, checked, a, msize, S, cnt, S - ct.loaded);
			break;
		}
		case 0x72: msize = 1; goto st;
		case 0x6a: msize = 2; goto st;
		case 0x62: msize = 4; goto st;
		case 0x7a: msize = 8;                                       /* STDW stores (u64)imm, sign-extended */
		st: {
			uint64_t a = D + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 1)))
				break;
			fault = mem_store(&re, checked, a, msize, IS, 0, 0);
			break;
		}
		default:                                                    /* :367-369 */
			fault = F_BAD_OPCODE;
			break;
		}
		if (fault)
			break;
		if (re.sdef && op == 0x85) /* a lookup result is an address (NULL is not) */
			taint[0] = p->helper_kind[imm] == ORACLE_HELPER_MAP_LOOKUP && reg[0] != 0;
		if (re.sdef && op == 0x18) {
			taint[d] = 0;
			for (uint32_t m = 0; m < p->nmaps; m++)
				taint[d] |= p->maps[m].handle == reg[d];
		}
		if (taken > 0) {
			uint32_t npc = pc + (uint32_t)(int32_t)off; /* pc += inst->offset (u32 wrap) */
			/* next state (idx + npc, npc + 1) == current (idx, pc) → the reference spins forever */
			if (npc == 0 && pc == 1) {
				fault = F_LOOP;
				break;
			}
			pc = npc;
		}
	}
done:
	if (fault)
		r0 = 0;
	if (fault_out)
		*fault_out = (uint8_t)fault;
	if (steps_out)
		*steps_out = steps;
	return r0;
}

/* Standard eBPF (ISA v3 without the v4 extensions), the semantics compilers target and the
 * Linux interpreter implements: sequential pc (a taken jump goes to pc + 1 + off), MOV64 moves
 * (imm sign-extended), NEG/NEG64 negate dst, arithmetic ARSH, DIV by zero = 0, MOD by zero =
 * dst (32-bit: truncated), the JMP32 class comparing the low 32 bits.  Everything else (memory
 * regions, helpers, LDDW, byte swaps, masked shift counts, fault codes) as in run_ref.
 * No reference implementation exists to pin this against: it is pinned
 * by hand-computed known-answer tests (tests/test_standard.py).  Loops: a lane may take
 * 2^20 backward jumps (taken, off < 0: the target is at or before the jump's own slot); the
 * next one faults F_LOOP (the device's budget, dprog.h DP_LOOP_BUDGET: the packet's run has no
 * other bound there). */
static uint64_t
run_std(const struct oracle_prog *p, int checked, uint8_t *pkt, uint64_t len, uint8_t *fault_out,
	uint64_t *steps_out)
{
	uint64_t reg[11];
	uint8_t stack[STACK_BYTES], sdef[STACK_BYTES];
	struct region_env re;
	uint64_t pc = 0, steps = 0, r0 = 0, back = 0;
	int fault = F_NONE;

	if (checked)
		memset(stack, p->stack_init, sizeof(stack));
	for (int i = 0; i < 11; i++)
		reg[i] = p->reg_init;
	reg[1] = (uint64_t)(uintptr_t)pkt;
	reg[10] = (uint64_t)(uintptr_t)(stack + STACK_BYTES);
	re.pkt_lo = (uint64_t)(uintptr_t)pkt;
	re.pkt_hi = re.pkt_lo + len;
	re.stk_lo = (uint64_t)(uintptr_t)stack;
	re.stk_hi = re.stk_lo + STACK_BYTES;
	re.sdef = p->track_undef ? sdef : NULL;
	if (re.sdef)
		memset(sdef, 0, sizeof(sdef));
	uint8_t taint[11] = {0};
	taint[1] = taint[10] = 1;
	re.p = p;
	re.map_hit = -1;
	struct cnt_track ct = {0, 0, 0, 0, 0, 0};

	for (;;) {
		if (pc >= p->nslots) {
			fault = F_SLOT;
			break;
		}
		steps++;
		const uint8_t *ip = p->insns + pc * 8;
		uint8_t op = ip[0];
		uint8_t d = ip[1] & 0x0f, s = ip[1] >> 4;
		int16_t off;
		int32_t imm;
		memcpy(&off, ip + 2, 2);
		memcpy(&imm, ip + 4, 4);
		pc++;
		const int jmp32 = (op & 7) == 6;
		if (!(valid_op(op) || op == 0xc3 || op == 0xdb ||
		      (jmp32 && valid_op((uint8_t)((op & 0xf8) | 5)) && op != 0x06 && op != 0x86 &&
		       op != 0x96))) {
			fault = F_BAD_OPCODE;
			break;
		}
		if (jmp32) { /* same register rules as the 64-bit compare */
			if (d >= 11 || ((op & 0x08) && s >= 11)) {
				fault = F_BAD_REG;
				break;
			}
		} else if ((uses_dst(op) && d >= 11) || (uses_src(op) && s >= 11)) {
			fault = F_BAD_REG;
			break;
		}
		uint64_t D = d < 11 ? reg[d] : 0, S = s < 11 ? reg[s] : 0;
		uint32_t D32 = (uint32_t)D, S32 = (uint32_t)S, I32 = (uint32_t)imm;
		uint64_t IS = (uint64_t)(int64_t)imm;
		int taken = -1;
		int msize = 0;
		if (re.sdef && (fault = taint_pre(&re, taint, jmp32 ? (uint8_t)((op & 0xf8) | 5) : op, d, s,
						   off, imm, reg, 1)))
			break;
		const int cnt = cnt_next(&ct, op, d, s, off, 1);
		if (jmp32) {
			const uint32_t B = (op & 0x08) ? S32 : I32;
			switch (op & 0xf0) {
			case 0x10: taken = D32 == B; break;
			case 0x20: taken = D32 > B; break;
			case 0x30: taken = D32 >= B; break;
			case 0x40: taken = (D32 & B) != 0; break;
			case 0x50: taken = D32 != B; break;
			case 0x60: taken = (int32_t)D32 > (int32_t)B; break;
			case 0x70: taken = (int32_t)D32 >= (int32_t)B; break;
			case 0xa0: taken = D32 < B; break;
			case 0xb0: taken = D32 <= B; break;
			case 0xc0: taken = (int32_t)D32 < (int32_t)B; break;
			case 0xd0: taken = (int32_t)D32 <= (int32_t)B; break;
			}
		} else switch (op) {
		/* where standard eBPF differs from the reference */
		case 0x84: reg[d] = (uint32_t)(0u - D32); break;
		case 0x87: reg[d] = 0 - D; break;
		case 0xbf: reg[d] = S; break;
		case 0xb7: reg[d] = IS; break;
		case 0xcc: reg[d] = (uint32_t)((int32_t)D32 >> (S32 & 31)); break;
		case 0xc4: reg[d] = (uint32_t)((int32_t)D32 >> (I32 & 31)); break;
		case 0xcf: reg[d] = (uint64_t)((int64_t)D >> (S & 63)); break;
		case 0xc7: reg[d] = (uint64_t)((int64_t)D >> (IS & 63)); break;
		case 0x3c: reg[d] = S32 ? D32 / S32 : 0; break;
		case 0x34: reg[d] = I32 ? D32 / I32 : 0; break;
		case 0x9c: reg[d] = S32 ? D32 % S32 : D32; break;
		case 0x94: reg[d] = I32 ? D32 % I32 : D32; break;
		case 0x3f: reg[d] = S ? D / S : 0; break;
		case 0x37: reg[d] = IS ? D / IS : 0; break;
		case 0x9f: reg[d] = S ? D % S : D; break;
		case 0x97: reg[d] = IS ? D % IS : D; break;
		/* the same as the reference */
		case 0x0c: reg[d] = (uint32_t)(D32 + S32); break;
		case 0x04: reg[d] = (uint32_t)(D32 + I32); break;
		case 0x1c: reg[d] = (uint32_t)(D32 - S32); break;
		case 0x14: reg[d] = (uint32_t)(D32 - I32); break;
		case 0x2c: reg[d] = (uint32_t)(D32 * S32); break;
		case 0x24: reg[d] = (uint32_t)(D32 * I32); break;
		case 0x4c: reg[d] = D32 | S32; break;
		case 0x44: reg[d] = D32 | I32; break;
		case 0x5c: reg[d] = D32 & S32; break;
		case 0x54: reg[d] = D32 & I32; break;
		case 0x6c: reg[d] = (uint32_t)(D32 << (S32 & 31)); break;
		case 0x64: reg[d] = (uint32_t)(D32 << (I32 & 31)); break;
		case 0x7c: reg[d] = D32 >> (S32 & 31); break;
		case 0x74: reg[d] = D32 >> (I32 & 31); break;
		case 0xac: reg[d] = D32 ^ S32; break;
		case 0xa4: reg[d] = D32 ^ I32; break;
		case 0xbc: reg[d] = S32; break;
		case 0xb4: reg[d] = I32; break;
		case 0xd4:
			if (imm == 16) reg[d] = (uint16_t)D;
			else if (imm == 32) reg[d] = D32;
			break;
		case 0xdc:
			if (imm == 16) reg[d] = bs16((uint16_t)D);
			else if (imm == 32) reg[d] = __builtin_bswap32(D32);
			else if (imm == 64) reg[d] = __builtin_bswap64(D);
			break;
		case 0x0f: reg[d] = D + S; break;
		case 0x07: reg[d] = D + IS; break;
		case 0x1f: reg[d] = D - S; break;
		case 0x17: reg[d] = D - IS; break;
		case 0x2f: reg[d] = D * S; break;
		case 0x27: reg[d] = D * IS; break;
		case 0x4f: reg[d] = D | S; break;
		case 0x47: reg[d] = D | IS; break;
		case 0x5f: reg[d] = D & S; break;
		case 0x57: reg[d] = D & IS; break;
		case 0x6f: reg[d] = D << (S & 63); break;
		case 0x67: reg[d] = D << (IS & 63); break;
		case 0x7f: reg[d] = D >> (S & 63); break;
		case 0x77: reg[d] = D >> (IS & 63); break;
		case 0xaf: reg[d] = D ^ S; break;
		case 0xa7: reg[d] = D ^ IS; break;
		case 0x05: taken = 1; break;
		case 0x1d: taken = D == S; break;
		case 0x15: taken = D == IS; break;
		case 0x2d: taken = D > S; break;
		case 0x25: taken = D > IS; break;
		case 0x3d: taken = D >= S; break;
		case 0x35: taken = D >= IS; break;
		case 0x4d: taken = (D & S) != 0; break;
		case 0x45: taken = (D & IS) != 0; break;
		case 0x5d: taken = D != S; break;
		case 0x55: taken = D != IS; break;
		case 0x6d: taken = (int64_t)D > (int64_t)S; break;
		case 0x65: taken = (int64_t)D > (int64_t)IS; break;
		case 0x7d: taken = (int64_t)D >= (int64_t)S; break;
		case 0x75: taken = (int64_t)D >= (int64_t)IS; break;
		case 0xad: taken = D < S; break;
		case 0xa5: taken = D < IS; break;
		case 0xbd: taken = D <= S; break;
		case 0xb5: taken = D <= IS; break;
		case 0xcd: taken = (int64_t)D < (int64_t)S; break;
		case 0xc5: taken = (int64_t)D < (int64_t)IS; break;
		case 0xdd: taken = (int64_t)D <= (int64_t)S; break;
		case 0xd5: taken = (int64_t)D <= (int64_t)IS; break;
		case 0x85: {
			uint64_t r = helper_call(&re, checked, imm, reg, &fault);
			if (!fault)
				reg[0] = r;
			break;
		}
		case 0x95: r0 = reg[0]; goto done;
		case 0x71: msize = 1; goto ldx;
		case 0x69: msize = 2; goto ldx;
		case 0x61: msize = 4; goto ldx;
		case 0x79: msize = 8;
		ldx: {
			uint64_t a = S + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 0)))
				break;
			reg[d] = checked && re.map_hit >= 0 ? load_mem(a, msize) : load_n(a, msize);
			cnt_load(&ct, d, s, off, msize, reg[d]);
			break;
		}
		case 0x18:
			if (pc >= p->nslots) { fault = F_SLOT; break; }
			{
				int32_t hi;
				memcpy(&hi, p->insns + pc * 8 + 4, 4);
				reg[d] = (uint64_t)I32 | ((uint64_t)(uint32_t)hi << 32);
			}
			pc++;
			break;
		case 0x73: msize = 1; goto stx;
		case 0x6b: msize = 2; goto stx;
		case 0x63: msize = 4; goto stx;
		case 0x7b: msize = 8;
		stx: {
			uint64_t a = D + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 1)))
				break;
			fault = mem_store(&re, checked, a, msize, S, cnt, S - ct.loaded);
			break;
		}
		case 0x72: msize = 1; goto st;
		case 0x6a: msize = 2; goto st;
		case 0x62: msize = 4; goto st;
		case 0x7a: msize = 8;
		st: {
			uint64_t a = D + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 1)))
				break;
			fault = mem_store(&re, checked, a, msize, IS, 0, 0);
			break;
		}
		/* XADD (standard eBPF, BPF_STX | BPF_XADD): *(u32 / u64 *)(dst + off) += src; imm 1
		 * (BPF_ADD | BPF_FETCH) also sets src to the old value.  In a batch: a counter update
		 * (ebpf_oracle.h). */
		case 0xc3: msize = 4; goto xadd;
		case 0xdb: msize = 8;
		xadd: {
			if (imm != 0 && imm != 1) {
				fault = F_BAD_OPCODE;
				break;
			}
			uint64_t a = D + (uint64_t)(int64_t)off;
			if (checked && (fault = check_access(&re, a, msize, 1)))
				break;
			const uint64_t old = checked && re.map_hit >= 0 ? load_mem(a, msize) : load_n(a, msize);
			fault = mem_store(&re, checked, a, msize, old + S, 1, S);
			if (!fault && imm == 1)
				reg[s] = old;
			break;
		}
		default:
			fault = F_BAD_OPCODE;
			break;
		}
		if (fault)
			break;
		if (re.sdef && op == 0x85) /* a lookup result is an address (NULL is not) */
			taint[0] = p->helper_kind[imm] == ORACLE_HELPER_MAP_LOOKUP && reg[0] != 0;
		if (re.sdef && op == 0x18) {
			taint[d] = 0;
			for (uint32_t m = 0; m < p->nmaps; m++)
				taint[d] |= p->maps[m].handle == reg[d];
		}
		if (taken > 0) {
			int64_t npc = (int64_t)pc + off;
			if (off < 0 && ++back > (1u << 20)) {
				fault = F_LOOP;
				break;
			}
			if (npc < 0) {
				fault = F_SLOT;
				break;
			}
			pc = (uint64_t)npc;
		}
	}
done:
	if (fault)
		r0 = 0;
	if (fault_out)
		*fault_out = (uint8_t)fault;
	if (steps_out)
		*steps_out = steps;
	return r0;
}

static inline uint64_t
run_one(const struct oracle_prog *p, int checked, uint8_t *pkt, uint64_t len, uint8_t *fault_out,
	uint64_t *steps_out)
{
	if (p->semantics == 1)
		return run_std(p, checked, pkt, len, fault_out, steps_out);
	return run_ref(p, checked, pkt, len, fault_out, steps_out);
}

/* Raw mode: the reference's own cost model — one switch per instruction, operands read inside
 * each case, raw pointer memory access, no fault checks (valid programs only; used for the
 * timed CPU baseline).  Same semantics as run_one(checked=0) on valid programs. */
#define RD (reg[ip->dst])
#define RS (reg[ip->src])
#define IMM32 ((uint32_t)ip->imm)
#define IMM64 ((uint64_t)(int64_t)ip->imm)
#define A32(expr) RD = (uint32_t)(expr); break
#define A64(expr) RD = (expr); break
#define JMPIF(c) if (c) pc += (uint32_t)(int32_t)ip->offset; break
#define MEMA(base) ((base) + (uint64_t)(int64_t)ip->offset)

struct raw_inst {
	uint8_t opcode;
	uint8_t dst : 4;
	uint8_t src : 4;
	int16_t offset;
	int32_t imm;
};

static uint64_t
run_raw(const struct oracle_prog *p, uint8_t *pkt, uint64_t *steps_out)
{
	uint64_t reg[11];
	uint8_t stack[STACK_BYTES];
	const struct raw_inst *ip = (const struct raw_inst *)p->insns;
	uint32_t pc = 0;
	uint64_t steps = 0;
	struct region_env re = {0, 0, 0, 0, p, NULL, -1};
	for (int i = 0; i < 11; i++)
		reg[i] = p->reg_init;
	reg[1] = (uint64_t)(uintptr_t)pkt;
	reg[10] = (uint64_t)(uintptr_t)(stack + STACK_BYTES);
	for (;;) {
		ip += pc++;
		steps++;
		switch (ip->opcode) {
		case 0x04: A32((uint32_t)RD + IMM32);
		case 0x0c: A32((uint32_t)RD + (uint32_t)RS);
		case 0x14: A32((uint32_t)RD - IMM32);
		case 0x1c: A32((uint32_t)RD - (uint32_t)RS);
		case 0x24: A32((uint32_t)RD * IMM32);
		case 0x2c: A32((uint32_t)RD * (uint32_t)RS);
		case 0x34: A32((uint32_t)RD / IMM32);
		case 0x3c: A32((uint32_t)RD / (uint32_t)RS);
		case 0x44: A32((uint32_t)RD | IMM32);
		case 0x4c: A32((uint32_t)RD | (uint32_t)RS);
		case 0x54: A32((uint32_t)RD & IMM32);
		case 0x5c: A32((uint32_t)RD & (uint32_t)RS);
		case 0x64: A32((uint32_t)RD << (IMM32 & 31));
		case 0x6c: A32((uint32_t)RD << (RS & 31));
		case 0x74: case 0xc4: A32((uint32_t)RD >> (IMM32 & 31));
		case 0x7c: case 0xcc: A32((uint32_t)RD >> (RS & 31));
		case 0x84: A32(0u - IMM32);
		case 0x94: A32((uint32_t)RD % IMM32);
		case 0x9c: A32((uint32_t)RD % (uint32_t)RS);
		case 0xa4: A32((uint32_t)RD ^ IMM32);
		case 0xac: A32((uint32_t)RD ^ (uint32_t)RS);
		case 0xb4: A32(IMM32);
		case 0xbc: A32((uint32_t)RS);
		case 0xd4:
			if (ip->imm == 16) RD = (uint16_t)RD;
			else if (ip->imm == 32) RD = (uint32_t)RD;
			break;
		case 0xdc:
			if (ip->imm == 16) RD = bs16((uint16_t)RD);
			else if (ip->imm == 32) RD = __builtin_bswap32((uint32_t)RD);
			else if (ip->imm == 64) RD = __builtin_bswap64(RD);
			break;
		case 0x07: case 0xb7: A64(RD + IMM64);
		case 0x0f: case 0xbf: A64(RD + RS);
		case 0x17: case 0x87: A64(RD - IMM64);
		case 0x1f: A64(RD - RS);
		case 0x27: A64(RD * IMM64);
		case 0x2f: A64(RD * RS);
		case 0x37: A64(RD / IMM64);
		case 0x3f: A64(RD / RS);
		case 0x47: A64(RD | IMM64);
		case 0x4f: A64(RD | RS);
		case 0x57: A64(RD & IMM64);
		case 0x5f: A64(RD & RS);
		case 0x67: A64(RD << (IMM64 & 63));
		case 0x6f: A64(RD << (RS & 63));
		case 0x77: case 0xc7: A64(RD >> (IMM64 & 63));
		case 0x7f: case 0xcf: A64(RD >> (RS & 63));
		case 0x97: A64(RD % IMM64);
		case 0x9f: A64(RD % RS);
		case 0xa7: A64(RD ^ IMM64);
		case 0xaf: A64(RD ^ RS);
		case 0x05: JMPIF(1);
		case 0x15: JMPIF(RD == IMM64);
		case 0x1d: JMPIF(RD == RS);
		case 0x25: JMPIF(RD > IMM64);
		case 0x2d: JMPIF(RD > RS);
		case 0x35: JMPIF(RD >= IMM64);
		case 0x3d: JMPIF(RD >= RS);
		case 0x45: JMPIF(RD & IMM64);
		case 0x4d: JMPIF(RD & RS);
		case 0x55: JMPIF(RD != IMM64);
		case 0x5d: JMPIF(RD != RS);
		case 0x65: JMPIF((int64_t)RD > (int64_t)IMM64);
		case 0x6d: JMPIF((int64_t)RD > (int64_t)RS);
		case 0x75: JMPIF((int64_t)RD >= (int64_t)IMM64);
		case 0x7d: JMPIF((int64_t)RD >= (int64_t)RS);
		case 0xa5: JMPIF(RD < IMM64);
		case 0xad: JMPIF(RD < RS);
		case 0xb5: JMPIF(RD <= IMM64);
		case 0xbd: JMPIF(RD <= RS);
		case 0xc5: JMPIF((int64_t)RD < (int64_t)IMM64);
		case 0xcd: JMPIF((int64_t)RD < (int64_t)RS);
		case 0xd5: JMPIF((int64_t)RD <= (int64_t)IMM64);
		case 0xdd: JMPIF((int64_t)RD <= (int64_t)RS);
		case 0x85: {
			int f = 0;
			reg[0] = helper_call(&re, 0, ip->imm, reg, &f);
			break;
		}
		case 0x95:
			*steps_out = steps;
			return reg[0];
		case 0x71: A64(load_n(MEMA(RS), 1));
		case 0x69: A64(load_n(MEMA(RS), 2));
		case 0x61: A64(load_n(MEMA(RS), 4));
		case 0x79: A64(load_n(MEMA(RS), 8));
		case 0x18:
			RD = (uint64_t)IMM32 | ((uint64_t)(uint32_t)(ip + 1)->imm << 32);
			pc++;
			break;
		case 0x73: store_n(MEMA(RD), 1, RS); break;
		case 0x6b: store_n(MEMA(RD), 2, RS); break;
		case 0x63: store_n(MEMA(RD), 4, RS); break;
		case 0x7b: store_n(MEMA(RD), 8, RS); break;
		case 0x72: store_n(MEMA(RD), 1, IMM64); break;
		case 0x6a: store_n(MEMA(RD), 2, IMM64); break;
		case 0x62: store_n(MEMA(RD), 4, IMM64); break;
		case 0x7a: store_n(MEMA(RD), 8, IMM64); break;
		default:
			*steps_out = steps;
			return 0;
		}
	}
}

uint64_t
oracle_run(const struct oracle_prog *p, uint8_t *pkt, uint64_t len, uint8_t *fault,
	   uint64_t *steps)
{
	if (p->checked)
		return run_one(p, 1, pkt, len, fault, steps);
	if (p->semantics == 1)
		return run_std(p, 0, pkt, len, fault, steps);
	uint64_t st = 0;
	uint64_t r = run_raw(p, pkt, &st);
	if (fault)
		*fault = 0;
	if (steps)
		*steps = st;
	return r;
}

/* ---- the slot graph of a standard-semantics program (ebpf_oracle.h: which programs loop, and
 * which read their counter updates back) ---- */

/* An opcode run_std executes (else F_BAD_OPCODE). */
static inline int
std_valid(uint8_t op)
{
	const int jmp32 = (op & 7) == 6;
	return valid_op(op) || op == 0xc3 || op == 0xdb ||
	       (jmp32 && valid_op((uint8_t)((op & 0xf8) | 5)) && op != 0x06 && op != 0x86 && op != 0x96);
}

/* A CALL of a helper the batch runs (lookup, update, delete; any other faults) */
static inline int
std_call_ok(const struct oracle_prog *p, int32_t imm)
{
	if (imm < 0 || imm >= 64)
		return 0;
	const uint8_t k = p->helper_kind[imm];
	return k == ORACLE_HELPER_MAP_LOOKUP || k == ORACLE_HELPER_MAP_UPDATE || k == ORACLE_HELPER_MAP_DELETE;
}

/* The slots execution may continue at after slot pc (both arms of a conditional jump; LDDW over
 * its second slot; none after EXIT or an invalid opcode), into succ[0..1]; *back = 1 when one of
 * them is a backward jump's target that makes a loop: a conditional jump with off < 0 whose
 * target is a slot of the program, or a JA with off < -1 (JA -1 jumps to itself forever: F_LOOP
 * at once, no loop body).  Returns the count. */
static int
std_succ(const struct oracle_prog *p, uint64_t pc, uint64_t succ[2], int *back)
{
	const uint8_t *ip = p->insns + pc * 8;
	const uint8_t op = ip[0], d = ip[1] & 0x0f, sr = ip[1] >> 4;
	int16_t off;
	int32_t imm;
	memcpy(&off, ip + 2, 2);
	memcpy(&imm, ip + 4, 4);
	*back = 0;
	if (!std_valid(op) || op == 0x95)
		return 0;
	if ((op == 0xc3 || op == 0xdb) && imm != 0 && imm != 1)
		return 0; /* F_BAD_OPCODE */
	if ((op & 7) == 6 ? (d >= 11 || ((op & 0x08) && sr >= 11))
			  : ((uses_dst(op) && d >= 11) || (uses_src(op) && sr >= 11)))
		return 0; /* F_BAD_REG */
	if (op == 0x85 && !std_call_ok(p, imm))
		return 0; /* F_HELPER / F_HELPER_UNSUPPORTED */
	if (op == 0x18) {
		succ[0] = pc + 2;
		return 1;
	}
	const int64_t target = (int64_t)pc + 1 + off;
	if (op == 0x05) {
		if (off == -1)
			return 0;
		*back = off < 0;
		if (target < 0)
			return 0;
		succ[0] = (uint64_t)target;
		return 1;
	}
	int n = 0;
	if (((op & 7) == 5 || (op & 7) == 6) && op != 0x85 && target >= 0 && (uint64_t)target < p->nslots) {
		*back = off < 0;
		succ[n++] = (uint64_t)target;
	}
	succ[n++] = pc + 1;
	return n;
}

/* Slots reachable from slot 0 (seen[], nslots bytes); returns 1 when a loop's backward jump is
 * among them. */
static int
std_reach(const struct oracle_prog *p, uint8_t *seen)
{
	uint64_t *work = malloc((p->nslots * 2 + 2) * sizeof(uint64_t)); /* (<= 2 pushes a slot) */
	size_t nw = 0;
	int loops = 0;
	memset(seen, 0, p->nslots);
	work[nw++] = 0;
	while (nw) {
		const uint64_t pc = work[--nw];
		if (pc >= p->nslots || seen[pc])
			continue;
		seen[pc] = 1;
		uint64_t sx[2];
		int back;
		const int k = std_succ(p, pc, sx, &back);
		loops |= back;
		for (int i = 0; i < k; i++)
			work[nw++] = sx[i];
	}
	free(work);
	return loops;
}

/* Does the program loop?  Only standard semantics has loops (a taken jump goes to pc + 1 + off;
 * the reference's stepping never lowers the slot, ebpf_interpreter.c:39,210).  Decided from the
 * program's own bytes: a backward jump (std_succ) reachable from slot 0. */
static int
prog_has_loops(const struct oracle_prog *p)
{
	if (p->semantics != 1 || p->nslots == 0)
		return 0;
	uint8_t *seen = malloc(p->nslots);
	const int loops = std_reach(p, seen);
	free(seen);
	return loops;
}

/* Registers a standard-semantics instruction reads (*rd) and writes (*wr), as bit masks: a CALL
 * reads its helper's arguments (lookup and delete r1, r2; update r1..r4) and writes r0, EXIT
 * reads r0, an invalid opcode nothing. */
static void
std_regs(const struct oracle_prog *p, const uint8_t *ip, uint16_t *rd, uint16_t *wr)
{
	const uint8_t op = ip[0], cls = op & 7;
	const uint16_t d = (uint16_t)(1u << (ip[1] & 0x0f)), s = (uint16_t)(1u << (ip[1] >> 4));
	*rd = *wr = 0;
	if (!std_valid(op))
		return;
	switch (cls) {
	case 0: /* LDDW */
		*wr = d;
		return;
	case 1: /* LDX */
		*rd = s;
		*wr = d;
		return;
	case 2: /* ST */
		*rd = d;
		return;
	case 3: /* STX, XADD (imm 1: src receives the old value) */
		*rd = d | s;
		if ((op == 0xc3 || op == 0xdb) && (int32_t)(ip[4] | ip[5] << 8 | ip[6] << 16 | (uint32_t)ip[7] << 24) == 1)
			*wr = s;
		return;
	case 5:
	case 6:
		if (op == 0x85) {
			int32_t imm;
			memcpy(&imm, ip + 4, 4);
			*rd = std_call_ok(p, imm) && p->helper_kind[imm] == ORACLE_HELPER_MAP_UPDATE ? 0x1e : 0x06;
			*wr = 1;
		} else if (op == 0x95) {
			*rd = 1;
		} else if (op != 0x05) {
			*rd = d | ((op & 0x08) ? s : 0);
		}
		return;
	default: /* ALU / ALU64: MOV writes only (reg: reads src), LE / BE read dst only */
		*wr = d;
		if ((op & 0xf0) == 0xb0)
			*rd = (op & 0x08) ? s : 0;
		else if ((op & 0xf0) == 0xd0 || (op & 0xf0) == 0x80)
			*rd = d;
		else
			*rd = d | ((op & 0x08) ? s : 0);
		return;
	}
}

/* The slot execution continues at from pc, JA chains followed (the counter idiom's "consecutive,
 * JA aside"); nslots when there is none. */
static uint64_t
std_next_exec(const struct oracle_prog *p, uint64_t pc)
{
	for (uint64_t hops = 0; pc < p->nslots && hops <= p->nslots; hops++) {
		const uint8_t *ip = p->insns + pc * 8;
		if (ip[0] != 0x05)
			return pc;
		int16_t off;
		memcpy(&off, ip + 2, 2);
		const int64_t t = (int64_t)pc + 1 + off;
		if (off == -1 || t < 0)
			return p->nslots;
		pc = (uint64_t)t;
	}
	return p->nslots;
}

/* Does a program with loops read its counter updates back (ebpf_oracle.h)?  From its bytes, on
 * the slot graph: a reachable XADD with BPF_FETCH (imm 1), or a reachable counter idiom —
 * LDX{W,DW} X = [P + off] (X != P), then (JA aside) ADD / SUB to X of an immediate or of a
 * register other than X (64-bit; 32-bit too for W), then STX [P + off] = X of the same width —
 * whose X is live after the STX (some path from there reads X before writing it; a backward
 * fixed point of std_regs over the graph). */
static int
prog_reads_counters(const struct oracle_prog *p)
{
	if (p->semantics != 1 || p->nslots == 0)
		return 0;
	const uint64_t n = p->nslots;
	uint8_t *seen = malloc(n);
	std_reach(p, seen);
	int rb = 0;
	for (uint64_t i = 0; i < n && !rb; i++) {
		const uint8_t *ip = p->insns + i * 8;
		rb = seen[i] && (ip[0] == 0xc3 || ip[0] == 0xdb) &&
		     (int32_t)(ip[4] | ip[5] << 8 | ip[6] << 16 | (uint32_t)ip[7] << 24) == 1;
	}
	uint16_t *lin = NULL;
	for (uint64_t a = 0; a < n && !rb; a++) {
		const uint8_t *la = p->insns + a * 8;
		const uint8_t X = la[1] & 0x0f, P = la[1] >> 4;
		if (!seen[a] || !(la[0] == 0x61 || la[0] == 0x79) || X == P)
			continue;
		const int size = la[0] == 0x79 ? 8 : 4;
		const uint64_t b = std_next_exec(p, a + 1);
		if (b >= n)
			continue;
		const uint8_t *lb = p->insns + b * 8;
		const uint8_t bs = lb[1] >> 4;
		int ok = 0;
		if ((lb[1] & 0x0f) == X) {
			switch (lb[0]) {
			case 0x07: case 0x17: ok = 1; break;
			case 0x0f: case 0x1f: ok = bs != X; break;
			case 0x04: case 0x14: ok = size == 4; break;
			case 0x0c: case 0x1c: ok = size == 4 && bs != X; break;
			}
		}
		if (!ok)
			continue;
		const uint64_t c = std_next_exec(p, b + 1);
		if (c >= n)
			continue;
		const uint8_t *lc = p->insns + c * 8;
		if (lc[0] != (size == 8 ? 0x7b : 0x63) || (lc[1] & 0x0f) != P || (lc[1] >> 4) != X ||
		    memcmp(lc + 2, la + 2, 2) != 0)
			continue;
		if (lin == NULL) { /* liveness, once: lin[i] = rd | (out & ~wr), out = OR of the successors' */
			lin = calloc(n, sizeof(uint16_t));
			for (int changed = 1; changed;) {
				changed = 0;
				for (uint64_t i = n; i-- > 0;) {
					uint16_t rd, wr, o = 0;
					std_regs(p, p->insns + i * 8, &rd, &wr);
					uint64_t sx[2];
					int back;
					const int k = std_succ(p, i, sx, &back);
					for (int j = 0; j < k; j++)
						if (sx[j] < n)
							o |= lin[sx[j]];
					const uint16_t in = (uint16_t)(rd | (o & ~wr));
					if (in != lin[i]) {
						lin[i] = in;
						changed = 1;
					}
				}
			}
		}
		uint64_t sx[2];
		int back;
		const int k = std_succ(p, c, sx, &back);
		for (int j = 0; j < k && !rb; j++)
			rb = sx[j] < n && ((lin[sx[j]] >> X) & 1);
	}
	free(lin);
	free(seen);
	return rb;
}

static int
wrec_cmp(const void *a, const void *b)
{
	const struct wrec *x = a, *y = b;
	if (x->pkt != y->pkt)
		return x->pkt < y->pkt ? -1 : 1;
	return x->seq < y->seq ? -1 : (x->seq > y->seq);
}

uint64_t
oracle_run_batch(const struct oracle_prog *p, uint8_t *data, const uint64_t *offsets,
		 uint64_t count, uint32_t stride, uint64_t *ret, uint8_t *faults, int nthreads)
{
	return oracle_run_batch_hlog(p, data, offsets, count, stride, ret, faults, nthreads, NULL, 0,
				     NULL);
}

uint64_t
oracle_run_batch_hlog(const struct oracle_prog *p, uint8_t *data, const uint64_t *offsets,
		      uint64_t count, uint32_t stride, uint64_t *ret, uint8_t *faults, int nthreads,
		      uint8_t *hlog, uint64_t hlog_cap, uint64_t *hlog_used)
{
	uint64_t total = 0;
	uint64_t hused = 0;
	if (nthreads <= 0)
		nthreads = 1;
	/* a checked run may store into map values: every thread keeps a log (and, batch mode, the
	 * packet's overlay); a sequential run writes in place on one thread */
	int writes = p->checked && p->nmaps > 0;
	for (int i = 0; i < 64; i++)
		writes |= p->helper_kind[i] == ORACLE_HELPER_MAP_UPDATE ||
			  p->helper_kind[i] == ORACLE_HELPER_MAP_DELETE;
	if (p->sequential)
		nthreads = 1;
	struct wlog *logs = writes ? calloc((size_t)nthreads, sizeof(struct wlog)) : NULL;
	const int loops = writes && prog_has_loops(p);
	const int rb = loops && prog_reads_counters(p);
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads) reduction(+ : total)
#endif
	{
#ifdef _OPENMP
		const int tid = omp_get_thread_num();
#else
		const int tid = 0;
#endif
		t_wlog = logs ? &logs[tid] : NULL;
		t_sequential = p->sequential;
		t_loops = loops;
		t_rb = rb;
		t_ovl = logs && p->checked && !p->sequential ? malloc(sizeof(struct ovl)) : NULL;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
		for (int64_t i = 0; i < (int64_t)count; i++) {
			uint8_t *pkt;
			uint64_t len;
			if (offsets) {
				pkt = data + offsets[i];
				len = offsets[i + 1] - offsets[i];
			} else {
				pkt = data + (uint64_t)i * stride;
				len = stride;
			}
			uint8_t f = 0;
			uint64_t st = 0;
			t_pkt = (uint64_t)i;
			t_seq = 0;
			t_writes = 0;
			t_words.n = 0;
			if (t_ovl)
				t_ovl->n = 0;
			size_t n0 = t_wlog ? t_wlog->n : 0;
			ret[i] = oracle_run(p, pkt, len, &f, &st);
			if (f && t_wlog) { /* a packet that faults leaves no write behind but its counter updates */
				size_t w = n0;
				for (size_t r = n0; r < t_wlog->n; r++)
					if (t_wlog->rec[r].kind == WR_ADD)
						t_wlog->rec[w++] = t_wlog->rec[r];
				t_wlog->n = w;
			}
			if (faults)
				faults[i] = f;
			total += st;
		}
		t_wlog = NULL;
		free(t_ovl);
		t_ovl = NULL;
		t_sequential = 0;
		t_loops = 0;
		t_rb = 0;
	}
	if (logs) {
		/* after the batch: every write in packet order (last writer of a key wins) */
		size_t n = 0;
		for (int t = 0; t < nthreads; t++)
			n += logs[t].n;
		struct wrec *all = malloc((n ? n : 1) * sizeof(*all));
		size_t k = 0;
		for (int t = 0; t < nthreads; t++)
			for (size_t j = 0; j < logs[t].n; j++) {
				all[k] = logs[t].rec[j];
				all[k].voff = (uint64_t)(uintptr_t)(logs[t].arena + logs[t].rec[j].voff);
				k++;
			}
		qsort(all, n, sizeof(*all), wrec_cmp);
		for (size_t j = 0; j < n; j++) {
			const struct oracle_map *m = &p->maps[all[j].map];
			if (all[j].kind != WR_HELPER) {
				const int sz = all[j].size;
				if (m->kind == ORACLE_MAP_HASH) {
					/* {u32 map, u32 op (3 store, 4 add) | size << 8 | offset << 16, key, data} */
					const uint64_t rs = 8 + m->key_size + m->value_size;
					if (hlog && hused + rs <= hlog_cap) {
						const uint32_t w = (all[j].kind == WR_ADD ? 4u : 3u) | (uint32_t)sz << 8 |
								   all[j].off << 16;
						memcpy(hlog + hused, &all[j].map, 4);
						memcpy(hlog + hused + 4, &w, 4);
						memcpy(hlog + hused + 8, m->keys + (uint64_t)m->key_size * all[j].key,
						       m->key_size);
						memset(hlog + hused + 8 + m->key_size, 0, m->value_size);
						memcpy(hlog + hused + 8 + m->key_size, &all[j].data, (size_t)sz);
					}
					hused += rs;
					continue;
				}
				uint8_t *at = m->data + all[j].off;
				const uint64_t v = all[j].kind == WR_ADD ? load_n((uint64_t)(uintptr_t)at, sz) + all[j].data
								       : all[j].data;
				store_n((uint64_t)(uintptr_t)at, sz, v);
				continue;
			}
			if (m->kind == ORACLE_MAP_HASH) {
				/* for the caller's replay: {u32 map, u32 op | flags << 8, key, value} */
				const uint64_t sz = 8 + m->key_size + m->value_size;
				if (hlog && hused + sz <= hlog_cap) {
					memcpy(hlog + hused, &all[j].map, 4);
					memcpy(hlog + hused + 4, &all[j].key, 4);
					memset(hlog + hused + 8, 0, m->key_size + m->value_size);
					memcpy(hlog + hused + 8, (const void *)(uintptr_t)all[j].voff,
					       (all[j].key & 0xff) == 1 ? m->key_size + m->value_size : m->key_size);
				}
				hused += sz;
				continue;
			}
			memcpy(m->data + (uint64_t)m->value_size * all[j].key,
			       (const void *)(uintptr_t)all[j].voff, m->value_size);
		}
		free(all);
		for (int t = 0; t < nthreads; t++) {
			free(logs[t].rec);
			free(logs[t].arena);
		}
		free(logs);
	}
	if (hlog_used)
		*hlog_used = hused;
	return total;
}
