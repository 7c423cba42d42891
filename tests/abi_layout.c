/* Prints sizeof/offsetof of the public ABI structs (compiled by tests/test_abi.py with gcc). */
#include <stddef.h>
#include <stdio.h>
#include "../include/ripplemq_engine.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
int main(void) {
  printf("rmq_config %zu\n", sizeof(rmq_config));
  printf("rmq_batch %zu\n", sizeof(rmq_batch));
  printf("rmq_fetch_req %zu\n", sizeof(rmq_fetch_req));
  printf("rmq_fetch_res %zu\n", sizeof(rmq_fetch_res));
  printf("rmq_partition_state %zu\n", sizeof(rmq_partition_state));
  printf("rmq_append_stats %zu\n", sizeof(rmq_append_stats));
  F(rmq_config, segment_bytes); F(rmq_config, max_batch_bytes); F(rmq_config, device); F(rmq_config, rank);
  F(rmq_config, pool_bytes); F(rmq_partition_state, segment_bytes);
  F(rmq_batch, pidx); F(rmq_batch, payload_bytes);
  F(rmq_fetch_res, count); F(rmq_fetch_res, status);
  F(rmq_partition_state, match); F(rmq_partition_state, replica_rank); F(rmq_partition_state, is_leader);
  F(rmq_partition_state, leader_commit);
  F(rmq_append_stats, rejected_no_space);
  return 0;
}
