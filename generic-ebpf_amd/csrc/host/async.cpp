// async.cpp — the host-buffer batch without blocking the caller (a NIC-ring
// or capture consumer fills its next segment while the GPU works on this one).  A job runs the
// same pipeline as ebpf_prog_run_batch (chunked H2D -> kernel -> D2H on the library's streams)
// on a worker thread bound to the caller's current device; the caller collects it with
// ebpf_batch_wait.  Jobs on one device share its staging pool, so several may be in flight.
#include <cerrno>
#include <new>
#include <string>
#include <thread>

#include "internal.h"

struct ebpf_batch_job {
	std::thread th;
	ebpf_pkt_batch batch;   // the caller's descriptor, copied (its buffers stay the caller's)
	ebpf_batch_stats stats;
	int rc = 0;
	std::string msg;
};

EBPF_EXPORT int
ebpf_prog_run_batch_async(struct ebpf_prog *ep, const struct ebpf_pkt_batch *batch, uint64_t *ret,
			  uint8_t *faults, struct ebpf_batch_job **job)
{
	if (job == nullptr || ep == nullptr || batch == nullptr || ret == nullptr) {
		set_last_error("prog, batch, ret or job is NULL");
		return EINVAL;
	}
	*job = nullptr;
	if (ebpf_gpu_device_count() == 0) {
		set_last_error("no GPU visible");
		return ENODEV;
	}
	ebpf_batch_job *j = new (std::nothrow) ebpf_batch_job;
	if (j == nullptr)
		return ENOMEM;
	j->batch = *batch;
	const int device = current_device();
	try {
		j->th = std::thread([j, ep, ret, faults, device] {
			j->rc = ebpf_gpu_set_device(device);
			if (j->rc == 0)
				j->rc = ebpf_prog_run_batch(ep, &j->batch, ret, faults, &j->stats);
			if (j->rc)
				j->msg = ebpf_gpu_last_error();
		});
	} catch (...) {
		delete j;
		set_last_error("no thread for the job");
		return EAGAIN;
	}
	*job = j;
	return 0;
}

EBPF_EXPORT int
ebpf_batch_wait(struct ebpf_batch_job *job, struct ebpf_batch_stats *stats)
{
	if (job == nullptr) {
		set_last_error("job is NULL");
		return EINVAL;
	}
	job->th.join();
	const int rc = job->rc;
	if (rc)
		set_last_error(job->msg);
	else if (stats)
		*stats = job->stats;
	delete job;
	return rc;
}
