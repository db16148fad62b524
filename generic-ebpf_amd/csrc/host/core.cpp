// core.cpp — library init, env, object lifetime and program objects.
//
//   ebpf_init / ebpf_deinit       ↔ Linux/ebpf/user/ebpf_linux_user.c:210-234 (epoch init; here
//                                   nothing to set up: device maps are read-only during a batch)
//   ebpf_env_create / _destroy    ↔ sys/dev/ebpf/ebpf_env.c:21-50
//   ebpf_obj_acquire / _release   ↔ sys/dev/ebpf/ebpf_obj.c:21-46
//   ebpf_prog_create / _destroy   ↔ sys/dev/ebpf/ebpf_prog.c:22-82 (same validation order and
//                                   errno values; prog_len is a byte count, :53,66)
#include "internal.h"

#include <new>

EBPF_EXPORT int
ebpf_init(void)
{
	return 0;
}

EBPF_EXPORT int
ebpf_deinit(void)
{
	return 0;
}

EBPF_EXPORT int
ebpf_env_create(struct ebpf_env **eep, const struct ebpf_config *ec)
{
	if (eep == nullptr || ec == nullptr)
		return EINVAL;
	struct ebpf_env *ee = new (std::nothrow) ebpf_env();
	if (ee == nullptr)
		return ENOMEM;
	ee->ec = ec;
	*eep = ee;
	return 0;
}

EBPF_EXPORT int
ebpf_env_destroy(struct ebpf_env *ee)
{
	if (ee == nullptr)
		return EINVAL; // the reference dereferences NULL here
	if (ee->ref.load() != 0)
		return EBUSY;
	delete ee;
	return 0;
}

void
env_acquire(struct ebpf_env *ee)
{
	ee->ref.fetch_add(1);
}

void
env_release(struct ebpf_env *ee)
{
	ee->ref.fetch_sub(1);
}

void
obj_init(struct ebpf_env *ee, struct ebpf_obj *eo)
{
	env_acquire(ee);
	eo->eo_ee = ee;
	eo->eo_ref.store(1);
}

EBPF_EXPORT void
ebpf_obj_acquire(struct ebpf_obj *eo)
{
	if (eo != nullptr)
		eo->eo_ref.fetch_add(1);
}

EBPF_EXPORT void
ebpf_obj_release(struct ebpf_obj *eo)
{
	if (eo == nullptr)
		return;
	if (eo->eo_ref.fetch_sub(1) == 1) {
		struct ebpf_env *ee = eo->eo_ee;
		eo->eo_dtor(eo); // frees the object
		env_release(ee);
	}
}

// ---------------------------------------------------------------------------- programs

static void
prog_dtor(struct ebpf_obj *eo)
{
	struct ebpf_prog *ep = reinterpret_cast<struct ebpf_prog *>(eo);
	for (uint32_t i = 0; i < ep->ndep_maps; i++)
		ebpf_obj_release(&ep->dep_maps[i]->eo);
	prog_release_device_state(ep);
	if (ep->xlated) // maps pinned by the translation (translate.cpp) so mirrors stay valid
		for (struct ebpf_map *m : ep->xlated->maps)
			ebpf_obj_release(&m->eo);
	free(ep->prog);
	delete ep;
}

EBPF_EXPORT int
ebpf_prog_create(struct ebpf_env *ee, struct ebpf_prog **epp, struct ebpf_prog_attr *attr)
{
	if (ee == nullptr || epp == nullptr || attr == nullptr || attr->type >= EBPF_TYPE_MAX ||
	    attr->prog == nullptr || attr->prog_len == 0)
		return EINVAL;
	const struct ebpf_prog_type *ept = ee->ec->prog_types[attr->type];
	if (ept == nullptr)
		return EINVAL;
	struct ebpf_prog *ep = new (std::nothrow) ebpf_prog();
	if (ep == nullptr)
		return ENOMEM;
	ep->prog = static_cast<struct ebpf_inst *>(malloc(attr->prog_len));
	if (ep->prog == nullptr) {
		delete ep;
		return ENOMEM;
	}
	obj_init(ee, &ep->eo);
	ep->eo.eo_type = EBPF_OBJ_TYPE_PROG;
	ep->eo.eo_dtor = prog_dtor;
	ep->ept = ept;
	ep->ndep_maps = 0;
	ep->prog_len = attr->prog_len;
	memcpy(ep->prog, attr->prog, attr->prog_len);
	memset(ep->dep_maps, 0, sizeof(ep->dep_maps));
	*epp = ep;
	return 0;
}

EBPF_EXPORT void
ebpf_prog_destroy(struct ebpf_prog *ep)
{
	if (ep == nullptr)
		return;
	ebpf_obj_release(&ep->eo);
}

// ebpf_prog_attach_map ↔ sys/dev/ebpf/ebpf_prog.c:84-109 (exported by the reference .so)
EBPF_EXPORT int
ebpf_prog_attach_map(struct ebpf_prog *ep, struct ebpf_map *em)
{
	if (ep == nullptr || em == nullptr)
		return EINVAL;
	if (ep->eo.eo_ee != em->eo.eo_ee)
		return EINVAL;
	if (ep->ndep_maps >= EBPF_PROG_MAX_ATTACHED_MAPS)
		return EBUSY;
	for (uint32_t i = 0; i < ep->ndep_maps; i++)
		if (ep->dep_maps[i] == em)
			return EEXIST;
	ebpf_obj_acquire(&em->eo);
	ep->dep_maps[ep->ndep_maps++] = em;
	return 0;
}
