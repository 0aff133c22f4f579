// Parameter-gradient reduce jobs (reduce_jobs.hip): the batch passed to reduce_jobs_kernel by value.
#pragma once

#include "common.hpp"

namespace cai {

// jobs per launch (the batch travels as kernel arguments, <= 4 KB): 32 -- a C2 backward's ~22 jobs in one launch
// instead of two (16 per launch until round 5)
#ifndef CAI_REDUCE_BATCH_MAX
#define CAI_REDUCE_BATCH_MAX 32   // A/B: 16
#endif
constexpr int CAI_REDUCE_BATCH = CAI_REDUCE_BATCH_MAX;

struct ReduceBatch {
    int n;
    int total;                         // blocks of the batch (the capped-grid kernel walks them)
    int start[CAI_REDUCE_BATCH];       // first block of each job
    cai_reduce_job jobs[CAI_REDUCE_BATCH];
};
static_assert(sizeof(ReduceBatch) <= 4096, "kernel argument block");

// blocks of a WGRAD job: its weight rows (reduce_jobs.hip's layout choice) + `nbias_blocks` bias blocks
int wgrad_job_blocks(int Ng, int Cq_pad, int k, int nbias_blocks);

// run `n` jobs (CAI_JOB_NONE entries skipped) in ceil(n / CAI_REDUCE_BATCH) launches
int launch_reduce_jobs(const cai_reduce_job* jobs, int n, hipStream_t st, int max_grid = 0);

}  // namespace cai
