// maps.cpp — generic map layer, array / percpu-array maps, helper descriptors.
//
//   ebpf_map_create ... ebpf_map_destroy ↔ sys/dev/ebpf/ebpf_map.c:28-174 (validation, dispatch
//                                          through emt->ops, manual env release on init failure)
//   eht_map_{lookup,update,delete}_elem  ↔ sys/dev/ebpf/ebpf_map.c:176-189
//   emt_array / emt_percpu_array         ↔ sys/dev/ebpf/ebpf_map_array.c:27-298
//   emt_hashtable / emt_percpu_hashtable ↔ sys/dev/ebpf/ebpf_map_hashtable.c (exported so
//        configs link; creating one returns EOPNOTSUPP — hash maps are the "next" row of
//        SURVEY.md §8(f), not part of this round's hot path)
//
// Every host-side write bumps em->version so device mirrors re-upload before the next batch.
// ebpf_map_lookup_elem hands out a writable pointer, so it marks the map dirty as well.
#include "internal.h"

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
	return static_cast<array_priv *>(em->data)[curcpu()].array + (uint64_t)em->value_size * k;
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
	memcpy(static_cast<array_priv *>(em->data)[curcpu()].array + (uint64_t)em->value_size * k,
	       value, em->value_size);
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
	return 0;
}

// ---- hash tables: not in this round's scope ----
int
hash_init_unsupported(struct ebpf_map *, struct ebpf_map_attr *)
{
	set_last_error("hashtable maps are not implemented by this engine yet");
	return EOPNOTSUPP;
}
void *hash_lookup_none(struct ebpf_map *, void *) { return nullptr; }
int hash_err4(struct ebpf_map *, void *, void *, uint64_t) { return EOPNOTSUPP; }
int hash_err2(struct ebpf_map *, void *) { return EOPNOTSUPP; }
int hash_err3(struct ebpf_map *, void *, void *) { return EOPNOTSUPP; }
void hash_deinit(struct ebpf_map *) {}

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
	{hash_init_unsupported, hash_lookup_none, hash_err4, hash_err2, hash_err3, hash_err4,
	 hash_err2, hash_err3, hash_deinit}};

EBPF_EXPORT const struct ebpf_map_type emt_percpu_hashtable = {
	"percpu_hashtable",
	{hash_init_unsupported, hash_lookup_none, hash_err4, hash_err2, hash_err3, hash_err4,
	 hash_err2, hash_err3, hash_deinit}};

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
	return em->emt->ops.lookup_elem(em, key);
}

EBPF_EXPORT int
ebpf_map_lookup_elem_from_user(struct ebpf_map *em, void *key, void *value)
{
	if (em == nullptr || key == nullptr || value == nullptr)
		return EINVAL;
	return em->emt->ops.lookup_elem_from_user(em, key, value);
}

EBPF_EXPORT int
ebpf_map_update_elem(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	if (em == nullptr || key == nullptr || value == nullptr || flags > EBPF_EXIST)
		return EINVAL;
	return em->emt->ops.update_elem(em, key, value, flags);
}

EBPF_EXPORT int
ebpf_map_update_elem_from_user(struct ebpf_map *em, void *key, void *value, uint64_t flags)
{
	if (em == nullptr)
		return EINVAL; // the reference performs no argument checks here (ebpf_map.c:112-123)
	return em->emt->ops.update_elem_from_user(em, key, value, flags);
}

EBPF_EXPORT int
ebpf_map_delete_elem(struct ebpf_map *em, void *key)
{
	if (em == nullptr || key == nullptr)
		return EINVAL;
	return em->emt->ops.delete_elem(em, key);
}

EBPF_EXPORT int
ebpf_map_delete_elem_from_user(struct ebpf_map *em, void *key)
{
	if (em == nullptr || key == nullptr)
		return EINVAL;
	return em->emt->ops.delete_elem_from_user(em, key);
}

EBPF_EXPORT int
ebpf_map_get_next_key_from_user(struct ebpf_map *em, void *key, void *next_key)
{
	// key == NULL is valid: "give me the first key" (ebpf_map.c:148-151)
	if (em == nullptr || next_key == nullptr)
		return EINVAL;
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
