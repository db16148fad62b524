// maps.cpp — generic map layer, array / percpu-array maps, helper descriptors.
//
//   ebpf_map_create ... ebpf_map_destroy ↔ sys/dev/ebpf/ebpf_map.c:28-174 (validation, dispatch
//                                          through emt->ops, manual env release on init failure)
//   eht_map_{lookup,update,delete}_elem  ↔ sys/dev/ebpf/ebpf_map.c:176-189
//   emt_array / emt_percpu_array         ↔ sys/dev/ebpf/ebpf_map_array.c:27-298
//   emt_hashtable / emt_percpu_hashtable ↔ sys/dev/ebpf/ebpf_map_hashtable.c:25-571 (host side:
//        power-of-two buckets, newest-first chains, preallocated elements with a per-CPU
//        spare for in-place replacement, jhash from csrc/jhash.h)
//
// Every host-side write bumps em->version so device mirrors re-upload before the next batch.
// ebpf_map_lookup_elem hands out a writable pointer, so it marks the map dirty as well.
#include "internal.h"
#include "../jhash.h"

#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <new>

namespace {

struct array_priv {
	uint8_t *array;
};

inline void
mark_dirty(struct ebpf_map *em)
{
	em->version.fetch_add(1);
}

uint16_t
ncpus()
{
	long n = sysconf(_SC_NPROCESSORS_ONLN); // ebpf_linux_user.c:77-81
	return n > 0 ? (uint16_t)n : 1;
}

uint16_t
curcpu()
{
	// ebpf_linux_user.c:83-112: first CPU of the calling thread's affinity mask
	cpu_set_t cpus;
	if (pthread_getaffinity_np(pthread_self(), sizeof(cpus), &cpus) != 0)
		return 0;
	for (int i = 0; i < CPU_SETSIZE && i < 256; i++)
		if (CPU_ISSET(i, &cpus))
			return (uint16_t)i;
	return 0;
}

// ---- array (ebpf_map_array.c:51-124, 173-211, 246-283) ----
int
array_init(struct ebpf_map *em, struct ebpf_map_attr *attr)
{
	array_priv *ma = static_cast<array_priv *>(calloc(1, sizeof(array_priv)));
	if (ma == nullptr)
		return ENOMEM;
	ma->array = static_cast<uint8_t *>(calloc(attr->max_entries, attr->value_size));
	if (ma->array == nullptr) {
		free(ma);
		return ENOMEM;
	}
	em->data = ma;
	em->percpu = false;
	return 0;
}

void
array_deinit(struct ebpf_map *em)
{
	array_priv *ma = static_cast<array_priv *>(em->data);
	free(ma->array);
	free(ma);
}

void *
array_lookup(struct ebpf_map *em, void *key)
{
	uint32_t k = *static_cast<uint32_t *>(key);
	if (k >= em->max_entries)
		return nullptr;
	mark_dirty(em);
	return static_cast<array_priv *>(em->data)->array + (uint64_t)em->value_size * k;
}

int
array_lookup_from_user(struct ebpf_map *em, void *key, void *value)
{
	uint32_t k = *static_cast<uint32_t *>(key);
	if (k >= em->max_entries)
		return EINVAL;
	memcpy(value, static_cast<array_priv *>(em->data)->array + (uint64_t)em->value_size * k,
	       em->value_size);
	return 0;
}

int
array_update_check(struct ebpf_map *em, void *key, uint64_t flags)
{
	if (flags & EBPF_NOEXIST) // every array slot always exists
		return EEXIST;
	if (*static_cast<uint32_t *>(key) >= em->max_entries)
		return EINVAL;
	return 0;
}

int
array_update(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	int error = array_update_check(em, key, flags);
	if (error != 0)
		return error;
	uint32_t k = *static_cast<uint32_t *>(key);
	memcpy(static_cast<array_priv *>(em->data)->array + (uint64_t)em->value_size * k, value,
	       em->value_size);
	mark_dirty(em);
	return 0;
}

int
array_delete(struct ebpf_map *, void *)
{
	return EINVAL; // array elements cannot be deleted
}

int
array_get_next_key(struct ebpf_map *em, void *key, void *next_key)
{
	uint32_t k = key ? *static_cast<uint32_t *>(key) : UINT32_MAX;
	uint32_t *nk = static_cast<uint32_t *>(next_key);
	if (k >= em->max_entries) {
		*nk = 0;
		return 0;
	}
	if (k == em->max_entries - 1)
		return ENOENT;
	*nk = k + 1;
	return 0;
}

// ---- percpu array (ebpf_map_array.c:38-49, 83-113, 141-171, 213-244) ----
int
percpu_init(struct ebpf_map *em, struct ebpf_map_attr *attr)
{
	uint16_t n = ncpus();
	array_priv *ma = static_cast<array_priv *>(calloc(n, sizeof(array_priv)));
	if (ma == nullptr)
		return ENOMEM;
	for (uint16_t i = 0; i < n; i++) {
		ma[i].array = static_cast<uint8_t *>(calloc(attr->max_entries, attr->value_size));
		if (ma[i].array == nullptr) {
			for (uint16_t j = 0; j < i; j++)
				free(ma[j].array);
			free(ma);
			return ENOMEM;
		}
	}
	em->data = ma;
	em->percpu = true;
	return 0;
}

void
percpu_deinit(struct ebpf_map *em)
{
	array_priv *ma = static_cast<array_priv *>(em->data);
	for (uint16_t i = 0; i < ncpus(); i++)
		free(ma[i].array);
	free(ma);
}

void *
percpu_lookup(struct ebpf_map *em, void *key)
{
	uint32_t k = *static_cast<uint32_t *>(key);
	if (k >= em->max_entries)
		return nullptr;
	mark_dirty(em); // the caller may write through the pointer
	return static_cast<array_priv *>(em->data)[curcpu() % ncpus()].array + (uint64_t)em->value_size * k;
}

int
percpu_lookup_from_user(struct ebpf_map *em, void *key, void *value)
{
	uint32_t k = *static_cast<uint32_t *>(key);
	if (k >= em->max_entries)
		return EINVAL;
	array_priv *ma = static_cast<array_priv *>(em->data);
	for (uint16_t i = 0; i < ncpus(); i++)
		memcpy(static_cast<uint8_t *>(value) + (uint64_t)em->value_size * i,
		       ma[i].array + (uint64_t)em->value_size * k, em->value_size);
	return 0;
}

int
percpu_update(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	int error = array_update_check(em, key, flags);
	if (error != 0)
		return error;
	uint32_t k = *static_cast<uint32_t *>(key);
	memcpy(static_cast<array_priv *>(em->data)[curcpu() % ncpus()].array + (uint64_t)em->value_size * k,
	       value, em->value_size);
	mark_dirty(em);
	return 0;
}

int
percpu_update_from_user(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	int error = array_update_check(em, key, flags);
	if (error != 0)
		return error;
	uint32_t k = *static_cast<uint32_t *>(key);
	array_priv *ma = static_cast<array_priv *>(em->data);
	for (uint16_t i = 0; i < ncpus(); i++)
		memcpy(ma[i].array + (uint64_t)em->value_size * k, value, em->value_size);
	mark_dirty(em);
	return 0;
}

// ---- hashtable / percpu hashtable (ebpf_map_hashtable.c) ----
// Elements live in one preallocated pool.  Free elements form a LIFO stack, like the
// reference's allocator (ebpf_allocator.c:80-144: blocks pushed in creation order, alloc and
// free at the head), which decides which percpu element (and its stale per-CPU values) a new
// key reuses.  Bucket chains are doubly linked, new elements at the head.
struct hash_priv {
	uint32_t key_size, value_size; // internal sizes, rounded up to 8 (:153-154)
	uint32_t nbuckets;             // max_entries rounded up to a power of two (:167)
	uint32_t nelems;               // pool size
	std::vector<int32_t> head;     // per bucket: first element or -1
	std::vector<int32_t> next, prev;
	std::vector<uint8_t> keys;     // nelems * key_size
	std::vector<uint8_t> vals;     // nelems * value_size (percpu: nelems * ncpus * value_size)
	std::vector<int32_t> free_stack; // back = head of the free list
	std::vector<int32_t> spare;    // non-percpu: per-CPU spare element (:207-224)
	uint16_t ncpu = 1;
	bool percpu = false;
	uint64_t nlive = 0;
	std::mutex lock; // one lock per map (the reference locks per bucket)

	uint8_t *key(int32_t e) { return keys.data() + (size_t)e * key_size; }
	uint8_t *val(int32_t e, uint16_t cpu = 0)
	{
		return vals.data() + ((size_t)e * (percpu ? ncpu : 1) + cpu) * value_size;
	}
	uint32_t bucket_of(const void *k, uint32_t ks) const
	{
		return ebpf_jhash(k, ks, 0) & (nbuckets - 1); // :58-62, :288
	}
	int32_t find(uint32_t b, const void *k, uint32_t ks)
	{
		for (int32_t e = head[b]; e >= 0; e = next[e])
			if (memcmp(key(e), k, ks) == 0)
				return e;
		return -1;
	}
	void link_head(uint32_t b, int32_t e)
	{
		prev[e] = -1;
		next[e] = head[b];
		if (head[b] >= 0)
			prev[head[b]] = e;
		head[b] = e;
	}
	void unlink(uint32_t b, int32_t e)
	{
		if (prev[e] >= 0)
			next[prev[e]] = next[e];
		else
			head[b] = next[e];
		if (next[e] >= 0)
			prev[next[e]] = prev[e];
		next[e] = prev[e] = -1;
	}
	int32_t alloc()
	{
		if (free_stack.empty())
			return -1;
		int32_t e = free_stack.back();
		free_stack.pop_back();
		return e;
	}
};

uint32_t
roundup_pow2(uint32_t x)
{
	uint32_t p = 1;
	while (p < x && p != 0)
		p <<= 1;
	return p;
}

int
hash_init(struct ebpf_map *em, struct ebpf_map_attr *attr)
{
	const bool pc = em->emt == &emt_percpu_hashtable;
	em->percpu = pc;
	const uint64_t ks = (attr->key_size + 7ull) & ~7ull, vs = (attr->value_size + 7ull) & ~7ull;
	if (ks + vs + 16 > UINT32_MAX) // :141-146 (16 = the element's list linkage)
		return E2BIG;
	hash_priv *h = new (std::nothrow) hash_priv();
	if (h == nullptr)
		return ENOMEM;
	try {
		h->key_size = (uint32_t)ks;
		h->value_size = (uint32_t)vs;
		h->percpu = pc;
		h->ncpu = ncpus();
		h->nbuckets = roundup_pow2(attr->max_entries);
		if (h->nbuckets == 0)
			throw std::bad_alloc();
		// pool: max_entries (+ one spare per CPU for non-percpu maps, :200-225)
		h->nelems = attr->max_entries + (pc ? 0u : h->ncpu);
		h->head.assign(h->nbuckets, -1);
		h->next.assign(h->nelems, -1);
		h->prev.assign(h->nelems, -1);
		h->keys.assign((size_t)h->nelems * h->key_size, 0);
		h->vals.assign((size_t)h->nelems * (pc ? h->ncpu : 1) * h->value_size, 0);
		h->free_stack.reserve(h->nelems);
		for (uint32_t e = 0; e < h->nelems; e++)
			h->free_stack.push_back((int32_t)e);
		if (!pc)
			for (uint16_t c = 0; c < h->ncpu; c++)
				h->spare.push_back(h->alloc());
	} catch (const std::bad_alloc &) {
		delete h;
		return ENOMEM;
	}
	em->data = h;
	return 0;
}

void
hash_deinit(struct ebpf_map *em)
{
	delete static_cast<hash_priv *>(em->data);
}

void *
hash_lookup(struct ebpf_map *em, void *key) // :285-301
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	int32_t e = h->find(h->bucket_of(key, em->key_size), key, em->key_size);
	if (e < 0)
		return nullptr;
	mark_dirty(em); // the caller may write through the pointer
	return h->val(e, h->percpu ? curcpu() % h->ncpu : 0);
}

int
hash_lookup_from_user(struct ebpf_map *em, void *key, void *value) // :303-342
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	int32_t e = h->find(h->bucket_of(key, em->key_size), key, em->key_size);
	if (e < 0)
		return ENOENT;
	if (!h->percpu) {
		memcpy(value, h->val(e), em->value_size);
		return 0;
	}
	for (uint16_t c = 0; c < h->ncpu; c++)
		memcpy(static_cast<uint8_t *>(value) + (size_t)em->value_size * c, h->val(e, c), em->value_size);
	return 0;
}

int
hash_check_flags(int32_t found, uint64_t flags) // :88-100
{
	if (found >= 0)
		return (flags & EBPF_NOEXIST) ? EEXIST : 0;
	return (flags & EBPF_EXIST) ? ENOENT : 0;
}

std::mutex &
hash_lock(struct ebpf_map *em)
{
	return static_cast<hash_priv *>(em->data)->lock;
}

int
hash_update(struct ebpf_map *em, void *key, void *value, uint64_t flags) // :344-390
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	std::lock_guard<std::mutex> g(hash_lock(em));
	const uint32_t b = h->bucket_of(key, em->key_size);
	const int32_t old = h->find(b, key, em->key_size);
	int error = hash_check_flags(old, flags);
	if (error)
		return error;
	int32_t ne;
	if (old >= 0) { // replace through this CPU's spare element, which the old one becomes
		const uint16_t c = curcpu() % h->ncpu;
		ne = h->spare[c];
		h->spare[c] = old;
	} else if ((ne = h->alloc()) < 0) {
		return EBUSY;
	}
	memcpy(h->key(ne), key, em->key_size);
	memcpy(h->val(ne), value, em->value_size);
	h->link_head(b, ne);
	if (old >= 0)
		h->unlink(b, old);
	else
		h->nlive++;
	mark_dirty(em);
	return 0;
}

int
hash_update_percpu_common(struct ebpf_map *em, void *key, void *value, uint64_t flags, bool all)
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	std::lock_guard<std::mutex> g(hash_lock(em));
	const uint32_t b = h->bucket_of(key, em->key_size);
	int32_t e = h->find(b, key, em->key_size);
	int error = hash_check_flags(e, flags);
	if (error)
		return error;
	const bool fresh = e < 0;
	if (fresh && (e = h->alloc()) < 0)
		return EBUSY;
	if (all) // from user: every CPU's copy (:433-473)
		for (uint16_t c = 0; c < h->ncpu; c++)
			memcpy(h->val(e, c), value, em->value_size);
	else // from a program: this CPU's copy (:392-431)
		memcpy(h->val(e, curcpu() % h->ncpu), value, em->value_size);
	if (fresh) {
		memcpy(h->key(e), key, em->key_size);
		h->link_head(b, e);
		h->nlive++;
	}
	mark_dirty(em);
	return 0;
}

int
hash_update_percpu(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	return hash_update_percpu_common(em, key, value, flags, false);
}

int
hash_update_percpu_from_user(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	return hash_update_percpu_common(em, key, value, flags, true);
}

int
hash_delete(struct ebpf_map *em, void *key) // :475-502: 0 whether or not the key existed
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	std::lock_guard<std::mutex> g(hash_lock(em));
	const uint32_t b = h->bucket_of(key, em->key_size);
	const int32_t e = h->find(b, key, em->key_size);
	if (e >= 0) {
		h->unlink(b, e);
		h->free_stack.push_back(e);
		h->nlive--;
		mark_dirty(em);
	}
	return 0;
}

int
hash_get_next_key(struct ebpf_map *em, void *key, void *next_key) // :504-541
{
	hash_priv *h = static_cast<hash_priv *>(em->data);
	std::lock_guard<std::mutex> g(hash_lock(em));
	uint32_t i = 0;
	if (key != nullptr) {
		const uint32_t b = h->bucket_of(key, em->key_size);
		const int32_t e = h->find(b, key, em->key_size);
		if (e >= 0) {
			if (h->next[e] >= 0) {
				memcpy(next_key, h->key(h->next[e]), em->key_size);
				return 0;
			}
			i = b + 1;
		}
	}
	for (; i < h->nbuckets; i++)
		if (h->head[i] >= 0) {
			memcpy(next_key, h->key(h->head[i]), em->key_size);
			return 0;
		}
	return ENOENT;
}

void
map_dtor(struct ebpf_obj *eo)
{
	struct ebpf_map *em = reinterpret_cast<struct ebpf_map *>(eo);
	{
		std::lock_guard<std::mutex> g(em->eo.eo_ee->lock);
		em->eo.eo_ee->maps.erase(em);
	}
	map_release_device_state(em);
	em->emt->ops.deinit(em);
	delete em;
}

} // namespace

uint8_t *
ebpf_map::array_storage() const
{
	if (emt != &emt_array || data == nullptr)
		return nullptr;
	return static_cast<array_priv *>(data)->array;
}

bool
ebpf_map::is_hashtable() const
{
	return emt == &emt_hashtable || emt == &emt_percpu_hashtable;
}

uint16_t
map_current_cpu()
{
	return (uint16_t)(curcpu() % ncpus());
}

const uint8_t *
map_array_image(struct ebpf_map *em, uint16_t cpu)
{
	if (em->emt == &emt_array)
		return static_cast<array_priv *>(em->data)->array;
	if (em->emt == &emt_percpu_array)
		return static_cast<array_priv *>(em->data)[cpu % ncpus()].array;
	return nullptr;
}

map_device_layout
map_device_layout_of(const struct ebpf_map *em)
{
	map_device_layout l;
	if (em->emt == &emt_array || em->emt == &emt_percpu_array) {
		l.bytes = (size_t)em->value_size * em->max_entries;
		l.slots = em->max_entries;
		return l;
	}
	if (!em->is_hashtable() || em->key_size == 0 || em->key_size > DP_HASH_MAX_KEY)
		return l;
	uint64_t need = dp_hash_value_off(em->key_size) + (uint64_t)em->value_size, stride = 16;
	uint32_t lg = 4;
	while (stride < need) {
		stride <<= 1;
		lg++;
	}
	// at most a quarter full: linear probing then ends within a slot or two almost always
	// (an unsuccessful search probes (1 + 1/(1-a)^2)/2 = 1.4 slots on average at a = 1/4);
	// an eighth full where the table stays within 1 GiB of HBM (C4H, 1M entries: 2% faster,
	// profiles/r02/v2occ/hash_slots_c4h.txt)
	uint64_t slots = 16, per = (uint64_t)em->max_entries * 8 * stride <= (1ull << 30) ? 8 : 4;
	if (const char *f = getenv("EBPF_HASH_SLOTS_PER_ENTRY")) // (A/B: table size vs probe length)
		per = std::max<uint64_t>(2, strtoull(f, nullptr, 0));
	while (slots < per * em->max_entries)
		slots <<= 1;
	if (lg > 31 || slots > (1ull << 31) || slots * stride > (1ull << 36))
		return l;
	l.bytes = (size_t)(slots * stride) + 16; // (+ the trailer, dprog.h dp_hash_trailer_off)
	l.slots = (uint32_t)slots;
	l.flags = DP_MAP_HASH | (lg << 16) | em->key_size;
	return l;
}

void
map_device_image(struct ebpf_map *em, std::vector<uint8_t> &out, uint16_t cpu)
{
	const map_device_layout l = map_device_layout_of(em);
	hash_priv *h = static_cast<hash_priv *>(em->data);
	std::lock_guard<std::mutex> g(hash_lock(em));
	out.assign(l.bytes, 0);
	const uint32_t lg = dp_hash_stride_log2(l.flags), mask = l.slots - 1;
	const uint32_t voff = dp_hash_value_off(em->key_size);
	for (uint32_t b = 0; b < h->nbuckets; b++)
		for (int32_t e = h->head[b]; e >= 0; e = h->next[e]) {
			const uint32_t hv = ebpf_jhash(h->key(e), em->key_size, 0);
			uint32_t i = hv & mask;
			while (out[((size_t)i << lg)] != 0)
				i = (i + 1) & mask;
			uint8_t *slot = out.data() + ((size_t)i << lg);
			const uint32_t used = 1;
			memcpy(slot, &used, 4);
			memcpy(slot + 4, &hv, 4);
			memcpy(slot + 8, h->key(e), em->key_size);
			memcpy(slot + voff, h->val(e, h->percpu ? cpu % h->ncpu : 0), em->value_size);
		}
	const uint32_t trailer[2] = {(uint32_t)h->nlive, em->max_entries};
	memcpy(out.data() + dp_hash_trailer_off(l.slots, l.flags), trailer, sizeof(trailer));
}

EBPF_EXPORT const struct ebpf_map_type emt_array = {
	"array",
	{array_init, array_lookup, array_update, array_delete, array_lookup_from_user, array_update,
	 array_delete, array_get_next_key, array_deinit}};

EBPF_EXPORT const struct ebpf_map_type emt_percpu_array = {
	"percpu_array",
	{percpu_init, percpu_lookup, percpu_update, array_delete, percpu_lookup_from_user,
	 percpu_update_from_user, array_delete, array_get_next_key, percpu_deinit}};

EBPF_EXPORT const struct ebpf_map_type emt_hashtable = {
	"hashtable",
	{hash_init, hash_lookup, hash_update, hash_delete, hash_lookup_from_user, hash_update,
	 hash_delete, hash_get_next_key, hash_deinit}};

EBPF_EXPORT const struct ebpf_map_type emt_percpu_hashtable = {
	"percpu_hashtable",
	{hash_init, hash_lookup, hash_update_percpu, hash_delete, hash_lookup_from_user,
	 hash_update_percpu_from_user, hash_delete, hash_get_next_key, hash_deinit}};

// ---------------------------------------------------------------------------- generic layer

EBPF_EXPORT int
ebpf_map_create(struct ebpf_env *ee, struct ebpf_map **emp, struct ebpf_map_attr *attr)
{
	if (ee == nullptr || emp == nullptr || attr == nullptr || attr->type >= EBPF_TYPE_MAX ||
	    attr->key_size == 0 || attr->value_size == 0 || attr->max_entries == 0)
		return EINVAL;
	const struct ebpf_map_type *emt = ee->ec->map_types[attr->type];
	if (emt == nullptr)
		return EINVAL;
	struct ebpf_map *em = new (std::nothrow) ebpf_map();
	if (em == nullptr)
		return ENOMEM;
	obj_init(ee, &em->eo);
	em->eo.eo_type = EBPF_OBJ_TYPE_MAP;
	em->eo.eo_dtor = map_dtor;
	em->emt = emt;
	em->key_size = attr->key_size;
	em->value_size = attr->value_size;
	em->max_entries = attr->max_entries;
	em->map_flags = attr->flags;
	em->percpu = false;
	em->data = nullptr;
	int error = emt->ops.init(em, attr);
	if (error != 0) {
		env_release(ee); // ebpf_map.c:59-70: init incomplete, undo the env ref by hand
		delete em;
		return error;
	}
	{
		std::lock_guard<std::mutex> g(ee->lock);
		ee->maps.insert(em);
	}
	*emp = em;
	return 0;
}

EBPF_EXPORT void *
ebpf_map_lookup_elem(struct ebpf_map *em, void *key)
{
	if (em == nullptr || key == nullptr)
		return nullptr;
	if (map_pull_device_writes(em) != 0)
		return nullptr; // (the device's writes could not be copied back: no stale value)
	return em->emt->ops.lookup_elem(em, key);
}

EBPF_EXPORT int
ebpf_map_lookup_elem_from_user(struct ebpf_map *em, void *key, void *value)
{
	if (em == nullptr || key == nullptr || value == nullptr)
		return EINVAL;
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.lookup_elem_from_user(em, key, value);
}

EBPF_EXPORT int
ebpf_map_update_elem(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	if (em == nullptr || key == nullptr || value == nullptr || flags > EBPF_EXIST)
		return EINVAL;
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.update_elem(em, key, value, flags);
}

EBPF_EXPORT int
ebpf_map_update_elem_from_user(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	if (em == nullptr)
		return EINVAL; // the reference performs no argument checks here (ebpf_map.c:112-123)
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.update_elem_from_user(em, key, value, flags);
}

EBPF_EXPORT int
ebpf_map_delete_elem(struct ebpf_map *em, void *key)
{
	if (em == nullptr || key == nullptr)
		return EINVAL;
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.delete_elem(em, key);
}

EBPF_EXPORT int
ebpf_map_delete_elem_from_user(struct ebpf_map *em, void *key)
{
	if (em == nullptr || key == nullptr)
		return EINVAL;
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.delete_elem_from_user(em, key);
}

EBPF_EXPORT int
ebpf_map_get_next_key_from_user(struct ebpf_map *em, void *key, void *next_key)
{
	// key == NULL is valid: "give me the first key" (ebpf_map.c:148-151)
	if (em == nullptr || next_key == nullptr)
		return EINVAL;
	if (map_pull_device_writes(em) != 0)
		return EIO;
	return em->emt->ops.get_next_key_from_user(em, key, next_key);
}

EBPF_EXPORT void
ebpf_map_destroy(struct ebpf_map *em)
{
	if (em == nullptr)
		return;
	ebpf_obj_release(&em->eo);
}

EBPF_EXPORT const struct ebpf_helper_type eht_map_lookup_elem = {
	"map_lookup_elem", reinterpret_cast<ebpf_helper_fn>(ebpf_map_lookup_elem)};
EBPF_EXPORT const struct ebpf_helper_type eht_map_update_elem = {
	"map_update_elem", reinterpret_cast<ebpf_helper_fn>(ebpf_map_update_elem)};
EBPF_EXPORT const struct ebpf_helper_type eht_map_delete_elem = {
	"map_delete_elem", reinterpret_cast<ebpf_helper_fn>(ebpf_map_delete_elem)};
