"""Application tuning knobs of the shipped cassandra and hdfs packages, one table each, and the
generator that keeps the package files in sync with the tables.

Each knob is one setting of the application's own configuration file -- a ``cassandra.yaml`` key
(Cassandra 3.11) or an ``hdfs-site.xml`` / ``core-site.xml`` property (Hadoop 2.x) -- with its type
and the application's default. From a table the generator writes, between marker lines:

* the package option (``universe/config.json``: ``cassandra.<key>`` / ``hdfs.<key>`` with type,
  default and description),
* the scheduler environment entry that carries it to every task (``marathon.json.mustache``:
  ``"TASKCFG_ALL_<ENV>": "{{cassandra.<key>}}"``; the scheduler's TaskEnvRouter hands
  ``TASKCFG_ALL_*`` to every pod without the prefix),
* the line of the config template that consumes it (``cassandra.yaml``: ``<key>: {{<ENV>}}``,
  ``hdfs-site.xml``: ``<property><name>..</name><value>{{<ENV>}}</value></property>``). A knob whose
  default is empty is left out of the file unless it is set (the application then picks its own
  value, e.g. Cassandra's auto-sized caches).

So a user of the package can set any of them at install or update time (``dcos package install
--options``, or ``TASKCFG_ALL_*`` on the scheduler app), and a change rolls out through the
service's update plan like any other configuration change.

    python -m dcos_commons_amd.tools.package_knobs          # rewrite the generated regions
    python -m dcos_commons_amd.tools.package_knobs --check  # exit 1 if a file is out of date
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
from collections import OrderedDict
from typing import Dict, List, NamedTuple, Optional, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Knob(NamedTuple):
    key: str                 # option key under the package section, and (upper-cased) the env name
    setting: str             # the application's own name for it
    type: str                # JSON schema type: integer | number | boolean | string
    default: object
    description: str
    env: Optional[str] = None   # env name without TASKCFG_ALL_ (default: PREFIX + KEY)


# -- cassandra.yaml (Cassandra 3.11 defaults) ------------------------------------------------------
_C = [
    ("hinted_handoff_enabled", "boolean", True, "Store hints for writes to unavailable replicas"),
    ("max_hint_window_in_ms", "integer", 10800000, "Stop generating hints for a node down this long"),
    ("hinted_handoff_throttle_in_kb", "integer", 1024, "Hint delivery throttle per delivery thread"),
    ("max_hints_delivery_threads", "integer", 2, "Threads delivering hints"),
    ("hints_flush_period_in_ms", "integer", 10000, "How often hints are flushed to disk"),
    ("max_hints_file_size_in_mb", "integer", 128, "Maximum size of one hints file"),
    ("batchlog_replay_throttle_in_kb", "integer", 1024, "Batchlog replay throttle"),
    ("disk_failure_policy", "string", "stop", "Policy on a data disk failure: die, stop_paranoid, stop, best_effort, ignore"),
    ("commit_failure_policy", "string", "stop", "Policy on a commit log failure: die, stop, stop_commit, ignore"),
    ("prepared_statements_cache_size_mb", "string", "", "Prepared statements cache size (empty: auto)"),
    ("thrift_prepared_statements_cache_size_mb", "string", "", "Thrift prepared statements cache size (empty: auto)"),
    ("key_cache_size_in_mb", "string", "", "Key cache size (empty: auto, min(5% of heap, 100 MB))"),
    ("key_cache_save_period", "integer", 14400, "Seconds between key cache saves"),
    ("row_cache_size_in_mb", "integer", 0, "Row cache size (0: disabled)"),
    ("row_cache_save_period", "integer", 0, "Seconds between row cache saves"),
    ("counter_cache_size_in_mb", "string", "", "Counter cache size (empty: auto)"),
    ("counter_cache_save_period", "integer", 7200, "Seconds between counter cache saves"),
    ("commitlog_sync", "string", "periodic", "Commit log sync mode: periodic or batch"),
    ("commitlog_sync_period_in_ms", "integer", 10000, "Periodic commit log sync interval"),
    ("commitlog_segment_size_in_mb", "integer", 32, "Commit log segment size"),
    ("commitlog_total_space_in_mb", "string", "", "Commit log space cap (empty: auto)"),
    ("concurrent_counter_writes", "integer", 32, "Concurrent counter writes"),
    ("concurrent_materialized_view_writes", "integer", 32, "Concurrent materialized view writes"),
    ("memtable_allocation_type", "string", "heap_buffers", "Memtable allocation: heap_buffers, offheap_buffers, offheap_objects"),
    ("memtable_heap_space_in_mb", "string", "", "Memtable on-heap space (empty: 1/4 of heap)"),
    ("memtable_offheap_space_in_mb", "string", "", "Memtable off-heap space (empty: 1/4 of heap)"),
    ("memtable_flush_writers", "integer", 2, "Memtable flush writer threads"),
    ("index_summary_capacity_in_mb", "string", "", "Index summary capacity (empty: 5% of heap)"),
    ("index_summary_resize_interval_in_minutes", "integer", 60, "Index summary resize interval"),
    ("trickle_fsync", "boolean", False, "fsync during sequential writes"),
    ("trickle_fsync_interval_in_kb", "integer", 10240, "Trickle fsync interval"),
    ("native_transport_max_threads", "integer", 128, "Native transport request threads"),
    ("native_transport_max_frame_size_in_mb", "integer", 256, "Largest native protocol frame"),
    ("native_transport_max_concurrent_connections", "integer", -1, "Native client connections (-1: unlimited)"),
    ("native_transport_max_concurrent_connections_per_ip", "integer", -1, "Native client connections per IP (-1: unlimited)"),
    ("rpc_keepalive", "boolean", True, "TCP keepalive on thrift connections"),
    ("rpc_server_type", "string", "sync", "Thrift server type: sync or hsha"),
    ("thrift_framed_transport_size_in_mb", "integer", 15, "Thrift frame size"),
    ("incremental_backups", "boolean", False, "Hard-link every flushed SSTable into backups/"),
    ("snapshot_before_compaction", "boolean", False, "Snapshot before each compaction"),
    ("auto_snapshot", "boolean", True, "Snapshot before a keyspace truncation or drop"),
    ("column_index_size_in_kb", "integer", 64, "Row index granularity"),
    ("column_index_cache_size_in_kb", "integer", 2, "Partition index entries kept in the key cache"),
    ("concurrent_compactors", "string", "", "Concurrent compactions (empty: min(disks, cores))"),
    ("sstable_preemptive_open_interval_in_mb", "integer", 50, "Early-open interval of compacting SSTables"),
    ("stream_throughput_outbound_megabits_per_sec", "integer", 200, "Outbound streaming throttle"),
    ("inter_dc_stream_throughput_outbound_megabits_per_sec", "integer", 200, "Cross-DC outbound streaming throttle"),
    ("read_request_timeout_in_ms", "integer", 5000, "Coordinator read timeout"),
    ("range_request_timeout_in_ms", "integer", 10000, "Coordinator range scan timeout"),
    ("write_request_timeout_in_ms", "integer", 2000, "Coordinator write timeout"),
    ("counter_write_request_timeout_in_ms", "integer", 5000, "Coordinator counter write timeout"),
    ("cas_contention_timeout_in_ms", "integer", 1000, "Lightweight transaction contention timeout"),
    ("truncate_request_timeout_in_ms", "integer", 60000, "Truncate timeout"),
    ("request_timeout_in_ms", "integer", 10000, "Default timeout of other operations"),
    ("slow_query_log_timeout_in_ms", "integer", 500, "Queries slower than this are logged"),
    ("cross_node_timeout", "boolean", False, "Use the coordinator's timestamp for request timeouts"),
    ("streaming_keep_alive_period_in_secs", "integer", 300, "Streaming keep-alive period"),
    ("phi_convict_threshold", "integer", 8, "Failure detector sensitivity"),
    ("dynamic_snitch_update_interval_in_ms", "integer", 100, "Dynamic snitch score update interval"),
    ("dynamic_snitch_reset_interval_in_ms", "integer", 600000, "Dynamic snitch score reset interval"),
    ("dynamic_snitch_badness_threshold", "number", 0.1, "Dynamic snitch badness threshold"),
    ("request_scheduler", "string", "org.apache.cassandra.scheduler.NoScheduler", "Client request scheduler"),
    ("internode_compression", "string", "dc", "Internode compression: all, dc, none"),
    ("inter_dc_tcp_nodelay", "boolean", False, "TCP_NODELAY on cross-DC connections"),
    ("tracetype_query_ttl", "integer", 86400, "TTL of query traces"),
    ("tracetype_repair_ttl", "integer", 604800, "TTL of repair traces"),
    ("enable_user_defined_functions", "boolean", False, "Allow Java user-defined functions"),
    ("enable_scripted_user_defined_functions", "boolean", False, "Allow scripted user-defined functions"),
    ("enable_materialized_views", "boolean", True, "Allow materialized views"),
    ("enable_sasi_indexes", "boolean", True, "Allow SASI indexes"),
    ("tombstone_warn_threshold", "integer", 1000, "Tombstones scanned by one query before a warning"),
    ("tombstone_failure_threshold", "integer", 100000, "Tombstones scanned by one query before it fails"),
    ("batch_size_warn_threshold_in_kb", "integer", 5, "Batch size that logs a warning"),
    ("batch_size_fail_threshold_in_kb", "integer", 50, "Batch size that fails the batch"),
    ("unlogged_batch_across_partitions_warn_threshold", "integer", 10, "Partitions of an unlogged batch before a warning"),
    ("compaction_large_partition_warning_threshold_mb", "integer", 100, "Partition size that logs a warning at compaction"),
    ("gc_warn_threshold_in_ms", "integer", 1000, "GC pause that logs a warning"),
    ("gc_log_threshold_in_ms", "integer", 200, "GC pause that is logged"),
    ("max_value_size_in_mb", "integer", 256, "Largest accepted value"),
    ("back_pressure_enabled", "boolean", False, "Coordinator back-pressure"),
    ("otc_coalescing_strategy", "string", "DISABLED", "Outbound message coalescing strategy"),
    ("otc_coalescing_window_us", "integer", 200, "Outbound coalescing window"),
    ("otc_coalescing_enough_coalesced_messages", "integer", 8, "Messages that end a coalescing window early"),
    ("otc_backlog_expiration_interval_ms", "integer", 200, "Outbound backlog expiration interval"),
    ("disk_optimization_strategy", "string", "ssd", "Disk optimization: ssd or spinning"),
    ("buffer_pool_use_heap_if_exhausted", "boolean", True, "Allocate on heap when the buffer pool is exhausted"),
    ("file_cache_size_in_mb", "string", "", "SSTable chunk cache (empty: min(512 MB, 1/4 of heap))"),
    ("cdc_enabled", "boolean", False, "Change data capture"),
    ("cdc_total_space_in_mb", "integer", 4096, "Space for CDC logs before writes to CDC tables fail"),
    ("cdc_free_space_check_interval_ms", "integer", 250, "CDC space recheck interval once the cap is hit"),
    ("start_native_transport", "boolean", True, "Serve the native (CQL) protocol"),
    ("commitlog_sync_batch_window_in_ms", "string", "", "Batch commit log window (batch sync only; empty: unset)"),
    ("key_cache_keys_to_save", "integer", 100, "Key cache keys saved (0: all)"),
    ("row_cache_keys_to_save", "integer", 100, "Row cache keys saved (0: all)"),
    ("counter_cache_keys_to_save", "integer", 100, "Counter cache keys saved (0: all)"),
    ("memtable_cleanup_threshold", "number", 0.11, "Memtable fill ratio that triggers a flush of the largest"),
    ("internode_authenticator", "string", "org.apache.cassandra.auth.AllowAllInternodeAuthenticator",
     "Authenticator of internode connections"),
    ("rpc_min_threads", "integer", 16, "Thrift request threads (minimum)"),
    ("rpc_max_threads", "integer", 2048, "Thrift request threads (maximum)"),
    ("rpc_send_buff_size_in_bytes", "integer", 16384, "Thrift socket send buffer"),
    ("rpc_recv_buff_size_in_bytes", "integer", 16384, "Thrift socket receive buffer"),
    ("windows_timer_interval", "integer", 1, "Windows timer resolution (ms; ignored elsewhere)"),
    ("repair_session_max_tree_depth", "integer", 18, "Merkle tree depth of a repair session"),
    ("listen_on_broadcast_address", "boolean", False, "Also listen on the broadcast address"),
    ("auto_bootstrap", "boolean", True, "Stream data to a new node when it joins"),
]

# -- hdfs-site.xml / core-site.xml (Hadoop 2.x defaults) -------------------------------------------
# (option key, property, type, default, description); the env is the key upper-cased
_H = [
    ("name_node_service_handler_count", "dfs.namenode.service.handler.count", "integer", 10, "NameNode service RPC handlers"),
    ("name_node_safemode_threshold_pct", "dfs.namenode.safemode.threshold-pct", "number", 0.999, "Fraction of blocks reported before safe mode ends"),
    ("name_node_safemode_extension", "dfs.namenode.safemode.extension", "integer", 30000, "Safe mode extension after the threshold (ms)"),
    ("name_node_safemode_min_datanodes", "dfs.namenode.safemode.min.datanodes", "integer", 0, "DataNodes required before safe mode ends"),
    ("name_node_heartbeat_recheck_interval", "dfs.namenode.heartbeat.recheck-interval", "integer", 300000, "Dead DataNode detection interval (ms)"),
    ("heartbeat_interval", "dfs.heartbeat.interval", "integer", 3, "DataNode heartbeat interval (s)"),
    ("name_node_checkpoint_period", "dfs.namenode.checkpoint.period", "integer", 3600, "Seconds between checkpoints"),
    ("name_node_checkpoint_txns", "dfs.namenode.checkpoint.txns", "integer", 1000000, "Transactions between checkpoints"),
    ("name_node_checkpoint_check_period", "dfs.namenode.checkpoint.check.period", "integer", 60, "Checkpoint trigger polling (s)"),
    ("name_node_num_checkpoints_retained", "dfs.namenode.num.checkpoints.retained", "integer", 2, "Image checkpoints kept"),
    ("name_node_num_extra_edits_retained", "dfs.namenode.num.extra.edits.retained", "integer", 1000000, "Extra edit transactions kept"),
    ("name_node_max_extra_edits_segments_retained", "dfs.namenode.max.extra.edits.segments.retained", "integer", 10000, "Extra edit log segments kept"),
    ("name_node_replication_min", "dfs.namenode.replication.min", "integer", 1, "Minimal block replication"),
    ("replication_max", "dfs.replication.max", "integer", 512, "Maximal block replication"),
    ("name_node_max_objects", "dfs.namenode.max.objects", "integer", 0, "Files + directories + blocks cap (0: none)"),
    ("name_node_decommission_interval", "dfs.namenode.decommission.interval", "integer", 30, "Decommission progress check (s)"),
    ("name_node_decommission_blocks_per_interval", "dfs.namenode.decommission.blocks.per.interval", "integer", 500000, "Blocks checked per decommission interval"),
    ("name_node_replication_interval", "dfs.namenode.replication.interval", "integer", 3, "Replication work computation period (s)"),
    ("name_node_accesstime_precision", "dfs.namenode.accesstime.precision", "integer", 3600000, "Access time precision (ms; 0 disables)"),
    ("name_node_fs_limits_max_component_length", "dfs.namenode.fs-limits.max-component-length", "integer", 255, "Longest path component"),
    ("name_node_fs_limits_max_directory_items", "dfs.namenode.fs-limits.max-directory-items", "integer", 1048576, "Most items in one directory"),
    ("name_node_fs_limits_min_block_size", "dfs.namenode.fs-limits.min-block-size", "integer", 1048576, "Smallest block size"),
    ("name_node_fs_limits_max_blocks_per_file", "dfs.namenode.fs-limits.max-blocks-per-file", "integer", 1048576, "Most blocks in one file"),
    ("name_node_stale_datanode_interval", "dfs.namenode.stale.datanode.interval", "integer", 30000, "DataNode considered stale after (ms)"),
    ("name_node_avoid_read_stale_datanode", "dfs.namenode.avoid.read.stale.datanode", "boolean", False, "Read from stale DataNodes last"),
    ("name_node_avoid_write_stale_datanode", "dfs.namenode.avoid.write.stale.datanode", "boolean", False, "Avoid writing to stale DataNodes"),
    ("name_node_write_stale_datanode_ratio", "dfs.namenode.write.stale.datanode.ratio", "number", 0.5, "Stale fraction above which writes use them again"),
    ("name_node_invalidate_work_pct_per_iteration", "dfs.namenode.invalidate.work.pct.per.iteration", "number", 0.32, "Invalidation work per heartbeat"),
    ("name_node_replication_work_multiplier_per_iteration", "dfs.namenode.replication.work.multiplier.per.iteration", "integer", 2, "Replication work per heartbeat"),
    ("name_node_top_enabled", "dfs.namenode.top.enabled", "boolean", True, "Top users metrics"),
    ("name_node_top_window_num_buckets", "dfs.namenode.top.window.num.buckets", "integer", 10, "Top users window buckets"),
    ("name_node_top_num_users", "dfs.namenode.top.num.users", "integer", 10, "Top users reported"),
    ("name_node_audit_log_async", "dfs.namenode.audit.log.async", "boolean", False, "Asynchronous audit log"),
    ("name_node_enable_retrycache", "dfs.namenode.enable.retrycache", "boolean", True, "Retry cache for non-idempotent RPCs"),
    ("name_node_retrycache_expirytime_millis", "dfs.namenode.retrycache.expirytime.millis", "integer", 600000, "Retry cache entry lifetime"),
    ("name_node_retrycache_heap_percent", "dfs.namenode.retrycache.heap.percent", "number", 0.03, "Heap share of the retry cache"),
    ("name_node_list_cache_pools_num_responses", "dfs.namenode.list.cache.pools.num.responses", "integer", 100, "Cache pools per listing"),
    ("name_node_list_cache_directives_num_responses", "dfs.namenode.list.cache.directives.num.responses", "integer", 100, "Cache directives per listing"),
    ("name_node_path_based_cache_refresh_interval_ms", "dfs.namenode.path.based.cache.refresh.interval.ms", "integer", 30000, "Cache directive rescan interval"),
    ("name_node_datanode_registration_ip_hostname_check", "dfs.namenode.datanode.registration.ip-hostname-check", "boolean", False, "Require resolvable DataNode addresses"),
    ("name_node_lifeline_handler_ratio", "dfs.namenode.lifeline.handler.ratio", "number", 0.1, "Lifeline RPC handler share"),
    ("name_node_quota_init_threads", "dfs.namenode.quota.init-threads", "integer", 4, "Quota initialisation threads"),
    ("name_node_edit_log_autoroll_multiplier_threshold", "dfs.namenode.edit.log.autoroll.multiplier.threshold", "number", 2.0, "Edit log roll threshold (x checkpoint txns)"),
    ("name_node_edit_log_autoroll_check_interval_ms", "dfs.namenode.edit.log.autoroll.check.interval.ms", "integer", 300000, "Edit log roll check interval"),
    ("name_node_name_cache_threshold", "dfs.namenode.name.cache.threshold", "integer", 10, "Name cache threshold"),
    ("name_node_delegation_key_update_interval", "dfs.namenode.delegation.key.update-interval", "integer", 86400000, "Delegation key update interval"),
    ("name_node_delegation_token_max_lifetime", "dfs.namenode.delegation.token.max-lifetime", "integer", 604800000, "Delegation token lifetime"),
    ("name_node_delegation_token_renew_interval", "dfs.namenode.delegation.token.renew-interval", "integer", 86400000, "Delegation token renewal interval"),
    ("name_node_inotify_max_events_per_rpc", "dfs.namenode.inotify.max.events.per.rpc", "integer", 1000, "inotify events per RPC"),
    ("name_node_reject_unresolved_dn_topology_mapping", "dfs.namenode.reject-unresolved-dn-topology-mapping", "boolean", False, "Reject DataNodes without a topology mapping"),
    ("name_node_resource_check_interval", "dfs.namenode.resource.check.interval", "integer", 5000, "Local storage check interval (ms)"),
    ("name_node_resource_du_reserved", "dfs.namenode.resource.du.reserved", "integer", 104857600, "Space kept free on NameNode volumes"),
    ("name_node_resource_checked_volumes_minimum", "dfs.namenode.resource.checked.volumes.minimum", "integer", 1, "Volumes that must have space"),
    ("name_node_startup_delay_block_deletion_sec", "dfs.namenode.startup.delay.block.deletion.sec", "integer", 0, "Delay block deletion after start-up"),
    ("name_node_acls_enabled", "dfs.namenode.acls.enabled", "boolean", False, "POSIX ACLs"),
    ("name_node_xattrs_enabled", "dfs.namenode.xattrs.enabled", "boolean", True, "Extended attributes"),
    ("name_node_fs_limits_max_xattrs_per_inode", "dfs.namenode.fs-limits.max-xattrs-per-inode", "integer", 32, "Extended attributes per inode"),
    ("name_node_fs_limits_max_xattr_size", "dfs.namenode.fs-limits.max-xattr-size", "integer", 16384, "Largest extended attribute"),
    ("name_node_blocks_per_postponedblocks_rescan", "dfs.namenode.blocks.per.postponedblocks.rescan", "integer", 10000, "Postponed blocks rescanned per iteration"),
    ("name_node_fslock_fair", "dfs.namenode.fslock.fair", "boolean", True, "Fair namesystem lock"),
    ("name_node_write_lock_reporting_threshold_ms", "dfs.namenode.write-lock-reporting-threshold-ms", "integer", 5000, "Long write lock holds are logged"),
    ("name_node_read_lock_reporting_threshold_ms", "dfs.namenode.read-lock-reporting-threshold-ms", "integer", 5000, "Long read lock holds are logged"),
    ("name_node_max_full_block_report_leases", "dfs.namenode.max.full.block.report.leases", "integer", 6, "Concurrent full block reports"),
    ("name_node_full_block_report_lease_length_ms", "dfs.namenode.full.block.report.lease.length.ms", "integer", 300000, "Full block report lease"),
    ("name_node_replication_consider_load", "dfs.namenode.replication.considerLoad", "boolean", True, "Consider DataNode load when placing replicas"),
    ("ha_tail_edits_period", "dfs.ha.tail-edits.period", "integer", 60, "Standby edit tailing period (s)"),
    ("ha_log_roll_period", "dfs.ha.log-roll.period", "integer", 120, "Active edit log roll period (s)"),
    ("ha_zkfc_nn_http_timeout_ms", "dfs.ha.zkfc.nn.http.timeout.ms", "integer", 20000, "ZKFC health check HTTP timeout"),
    ("ha_standby_checkpoints", "dfs.ha.standby.checkpoints", "boolean", True, "The standby NameNode checkpoints"),
    ("image_compression_codec", "dfs.image.compression.codec", "string", "org.apache.hadoop.io.compress.DefaultCodec", "fsimage compression codec"),
    ("image_transfer_timeout", "dfs.image.transfer.timeout", "integer", 60000, "fsimage transfer timeout"),
    ("image_transfer_bandwidth_per_sec", "dfs.image.transfer.bandwidthPerSec", "integer", 0, "fsimage transfer throttle (0: none)"),
    ("image_transfer_chunksize", "dfs.image.transfer.chunksize", "integer", 65536, "fsimage transfer chunk size"),
    ("blocksize", "dfs.blocksize", "integer", 134217728, "Default block size of new files"),
    ("block_scanner_volume_bytes_per_second", "dfs.block.scanner.volume.bytes.per.second", "integer", 1048576, "Block scanner throttle per volume"),
    ("bytes_per_checksum", "dfs.bytes-per-checksum", "integer", 512, "Bytes per checksum"),
    ("checksum_type", "dfs.checksum.type", "string", "CRC32C", "Checksum type"),
    ("client_write_packet_size", "dfs.client-write-packet-size", "integer", 65536, "Client write packet size"),
    ("client_block_write_retries", "dfs.client.block.write.retries", "integer", 3, "Block write retries"),
    ("client_block_write_replace_datanode_on_failure_enable", "dfs.client.block.write.replace-datanode-on-failure.enable", "boolean", True, "Replace failed DataNodes in a write pipeline"),
    ("client_block_write_replace_datanode_on_failure_policy", "dfs.client.block.write.replace-datanode-on-failure.policy", "string", "DEFAULT", "Pipeline DataNode replacement policy"),
    ("client_block_write_replace_datanode_on_failure_best_effort", "dfs.client.block.write.replace-datanode-on-failure.best-effort", "boolean", False, "Continue when no replacement DataNode is found"),
    ("client_read_shortcircuit", "dfs.client.read.shortcircuit", "boolean", False, "Short-circuit local reads (needs dfs.domain.socket.path)"),
    ("client_read_shortcircuit_streams_cache_size", "dfs.client.read.shortcircuit.streams.cache.size", "integer", 256, "Short-circuit file descriptor cache size"),
    ("client_read_shortcircuit_streams_cache_expiry_ms", "dfs.client.read.shortcircuit.streams.cache.expiry.ms", "integer", 300000, "Short-circuit file descriptor cache expiry"),
    ("client_socket_timeout", "dfs.client.socket-timeout", "integer", 60000, "Client socket timeout"),
    ("client_failover_max_attempts", "dfs.client.failover.max.attempts", "integer", 15, "Client failover attempts"),
    ("client_failover_sleep_base_millis", "dfs.client.failover.sleep.base.millis", "integer", 500, "Client failover backoff base"),
    ("client_failover_sleep_max_millis", "dfs.client.failover.sleep.max.millis", "integer", 15000, "Client failover backoff cap"),
    ("client_retry_policy_enabled", "dfs.client.retry.policy.enabled", "boolean", False, "Client RPC retry policy"),
    ("client_use_datanode_hostname", "dfs.client.use.datanode.hostname", "boolean", False, "Clients connect to DataNodes by hostname"),
    ("client_context", "dfs.client.context", "string", "default", "Client cache context name"),
    ("client_mmap_enabled", "dfs.client.mmap.enabled", "boolean", True, "Zero-copy reads through mmap"),
    ("client_mmap_cache_size", "dfs.client.mmap.cache.size", "integer", 256, "mmap regions cached"),
    ("client_mmap_cache_timeout_ms", "dfs.client.mmap.cache.timeout.ms", "integer", 3600000, "mmap cache expiry"),
    ("client_short_circuit_replica_stale_threshold_ms", "dfs.client.short.circuit.replica.stale.threshold.ms", "integer", 1800000, "Short-circuit replica staleness"),
    ("data_node_handler_count", "dfs.datanode.handler.count", "integer", 10, "DataNode RPC handlers"),
    ("data_node_max_transfer_threads", "dfs.datanode.max.transfer.threads", "integer", 4096, "DataNode transfer threads"),
    ("data_node_balance_bandwidth_per_sec", "dfs.datanode.balance.bandwidthPerSec", "integer", 1048576, "Balancer bandwidth per DataNode"),
    ("data_node_balance_max_concurrent_moves", "dfs.datanode.balance.max.concurrent.moves", "integer", 5, "Concurrent balancer moves"),
    ("data_node_du_reserved", "dfs.datanode.du.reserved", "integer", 0, "Space kept free per DataNode volume"),
    ("data_node_failed_volumes_tolerated", "dfs.datanode.failed.volumes.tolerated", "integer", 0, "Failed volumes before the DataNode stops"),
    ("data_node_directoryscan_interval", "dfs.datanode.directoryscan.interval", "integer", 21600, "Directory scan interval (s)"),
    ("data_node_directoryscan_threads", "dfs.datanode.directoryscan.threads", "integer", 1, "Directory scan threads"),
    ("data_node_scan_period_hours", "dfs.datanode.scan.period.hours", "integer", 504, "Block scanner period"),
    ("data_node_readahead_bytes", "dfs.datanode.readahead.bytes", "integer", 4194304, "Read-ahead"),
    ("data_node_drop_cache_behind_reads", "dfs.datanode.drop.cache.behind.reads", "boolean", False, "Drop page cache behind reads"),
    ("data_node_drop_cache_behind_writes", "dfs.datanode.drop.cache.behind.writes", "boolean", False, "Drop page cache behind writes"),
    ("data_node_sync_behind_writes", "dfs.datanode.sync.behind.writes", "boolean", False, "Sync behind writes"),
    ("data_node_use_datanode_hostname", "dfs.datanode.use.datanode.hostname", "boolean", False, "DataNodes connect to each other by hostname"),
    ("data_node_socket_write_timeout", "dfs.datanode.socket.write.timeout", "integer", 480000, "DataNode socket write timeout"),
    ("data_node_cache_revocation_timeout_ms", "dfs.datanode.cache.revocation.timeout.ms", "integer", 900000, "Cache revocation timeout"),
    ("data_node_cache_revocation_polling_ms", "dfs.datanode.cache.revocation.polling.ms", "integer", 500, "Cache revocation polling"),
    ("data_node_max_locked_memory", "dfs.datanode.max.locked.memory", "integer", 0, "Memory for the DataNode's block cache"),
    ("data_node_slow_io_warning_threshold_ms", "dfs.datanode.slow.io.warning.threshold.ms", "integer", 300, "Slow I/O warning threshold"),
    ("data_node_block_pinning_enabled", "dfs.datanode.block-pinning.enabled", "boolean", False, "Block pinning"),
    ("data_node_bp_ready_timeout", "dfs.datanode.bp-ready.timeout", "integer", 20, "Block pool ready timeout (s)"),
    ("data_node_cached_dfsused_check_interval_ms", "dfs.datanode.cached-dfsused.check.interval.ms", "integer", 600000, "Cached dfsUsed validity"),
    ("data_node_fsdatasetcache_max_threads_per_volume", "dfs.datanode.fsdatasetcache.max.threads.per.volume", "integer", 4, "Cache threads per volume"),
    ("data_node_transfer_socket_send_buffer_size", "dfs.datanode.transfer.socket.send.buffer.size", "integer", 131072, "Transfer socket send buffer"),
    ("data_node_transfer_socket_recv_buffer_size", "dfs.datanode.transfer.socket.recv.buffer.size", "integer", 131072, "Transfer socket receive buffer"),
    ("data_node_lazywriter_interval_sec", "dfs.datanode.lazywriter.interval.sec", "integer", 60, "Lazy persist writer interval"),
    ("qjournal_start_segment_timeout_ms", "dfs.qjournal.start-segment.timeout.ms", "integer", 20000, "Quorum journal start-segment timeout"),
    ("qjournal_prepare_recovery_timeout_ms", "dfs.qjournal.prepare-recovery.timeout.ms", "integer", 120000, "Quorum journal prepare-recovery timeout"),
    ("qjournal_accept_recovery_timeout_ms", "dfs.qjournal.accept-recovery.timeout.ms", "integer", 120000, "Quorum journal accept-recovery timeout"),
    ("qjournal_finalize_segment_timeout_ms", "dfs.qjournal.finalize-segment.timeout.ms", "integer", 120000, "Quorum journal finalize-segment timeout"),
    ("qjournal_select_input_streams_timeout_ms", "dfs.qjournal.select-input-streams.timeout.ms", "integer", 20000, "Quorum journal select-input-streams timeout"),
    ("qjournal_get_journal_state_timeout_ms", "dfs.qjournal.get-journal-state.timeout.ms", "integer", 120000, "Quorum journal get-state timeout"),
    ("qjournal_new_epoch_timeout_ms", "dfs.qjournal.new-epoch.timeout.ms", "integer", 120000, "Quorum journal new-epoch timeout"),
    ("qjournal_write_txns_timeout_ms", "dfs.qjournal.write-txns.timeout.ms", "integer", 20000, "Quorum journal write timeout"),
    ("qjournal_queued_edits_limit_mb", "dfs.qjournal.queued-edits.limit.mb", "integer", 10, "Queued edits per JournalNode"),
    ("encrypt_data_transfer", "dfs.encrypt.data.transfer", "boolean", False, "Encrypt block data transfer"),
    ("encrypt_data_transfer_algorithm", "dfs.encrypt.data.transfer.algorithm", "string", "", "Data transfer encryption algorithm (3des, rc4)"),
    ("encrypt_data_transfer_cipher_key_bitlength", "dfs.encrypt.data.transfer.cipher.key.bitlength", "integer", 128, "Data transfer cipher key length"),
    ("encrypt_data_transfer_cipher_suites", "dfs.encrypt.data.transfer.cipher.suites", "string", "", "Data transfer cipher suites (AES/CTR/NoPadding)"),
    ("data_transfer_protection", "dfs.data.transfer.protection", "string", "", "SASL data transfer protection: authentication, integrity, privacy"),
    ("permissions_superusergroup", "dfs.permissions.superusergroup", "string", "supergroup", "Super-user group"),
    ("cluster_administrators", "dfs.cluster.administrators", "string", "", "ACL of cluster administrators"),
    ("webhdfs_enabled", "dfs.webhdfs.enabled", "boolean", True, "WebHDFS REST API"),
    ("webhdfs_rest_csrf_enabled", "dfs.webhdfs.rest-csrf.enabled", "boolean", False, "WebHDFS CSRF protection"),
    ("webhdfs_ugi_expire_after_access", "dfs.webhdfs.ugi.expire.after.access", "integer", 600000, "WebHDFS UGI cache expiry"),
    ("user_home_dir_prefix", "dfs.user.home.dir.prefix", "string", "/user", "Home directory prefix"),
    ("storage_policy_enabled", "dfs.storage.policy.enabled", "boolean", True, "Storage policies"),
    ("stream_buffer_size", "dfs.stream-buffer-size", "integer", 4096, "Stream buffer size"),
    ("domain_socket_path", "dfs.domain.socket.path", "string", "", "UNIX domain socket for short-circuit reads"),
    ("block_access_key_update_interval", "dfs.block.access.key.update.interval", "integer", 600, "Block access key update interval (min)"),
    ("block_access_token_lifetime", "dfs.block.access.token.lifetime", "integer", 600, "Block access token lifetime (min)"),
    ("default_chunk_view_size", "dfs.default.chunk.view.size", "integer", 32768, "Bytes shown in the browser"),
    ("blockreport_interval_msec", "dfs.blockreport.intervalMsec", "integer", 21600000, "Full block report interval"),
    ("blockreport_initial_delay", "dfs.blockreport.initialDelay", "integer", 0, "First block report delay (s)"),
    ("blockreport_split_threshold", "dfs.blockreport.split.threshold", "integer", 1000000, "Blocks above which reports are split per volume"),
    ("cachereport_interval_msec", "dfs.cachereport.intervalMsec", "integer", 10000, "Cache report interval"),
    ("block_misreplication_processing_limit", "dfs.block.misreplication.processing.limit", "integer", 10000, "Mis-replicated blocks processed per run"),
    ("block_replicator_classname", "dfs.block.replicator.classname", "string",
     "org.apache.hadoop.hdfs.server.blockmanagement.BlockPlacementPolicyDefault", "Block placement policy"),
    ("xframe_enabled", "dfs.xframe.enabled", "boolean", True, "X-Frame-Options header on the web UIs"),
    ("xframe_value", "dfs.xframe.value", "string", "SAMEORIGIN", "X-Frame-Options value"),
    ("http_client_retry_policy_enabled", "dfs.http.client.retry.policy.enabled", "boolean", False, "WebHDFS client retry policy"),
    ("client_https_need_auth", "dfs.client.https.need-auth", "boolean", False, "Require client certificates on HTTPS"),
]

_CORE = [
    ("io_file_buffer_size", "io.file.buffer.size", "integer", 4096, "I/O buffer size"),
    ("fs_trash_interval", "fs.trash.interval", "integer", 0, "Minutes deleted files stay in the trash (0: no trash)"),
    ("fs_trash_checkpoint_interval", "fs.trash.checkpoint.interval", "integer", 0, "Minutes between trash checkpoints"),
    ("fs_df_interval", "fs.df.interval", "integer", 60000, "Disk usage statistics refresh"),
    ("fs_du_interval", "fs.du.interval", "integer", 600000, "Space used refresh"),
    ("ipc_client_connect_max_retries", "ipc.client.connect.max.retries", "integer", 10, "IPC connection retries"),
    ("ipc_client_connect_retry_interval", "ipc.client.connect.retry.interval", "integer", 1000, "IPC connection retry interval"),
    ("ipc_client_connect_timeout", "ipc.client.connect.timeout", "integer", 20000, "IPC connection timeout"),
    ("ipc_client_connect_max_retries_on_timeouts", "ipc.client.connect.max.retries.on.timeouts", "integer", 45, "IPC retries on connection timeouts"),
    ("ipc_client_connection_maxidletime", "ipc.client.connection.maxidletime", "integer", 10000, "Idle IPC connection lifetime"),
    ("ipc_client_idlethreshold", "ipc.client.idlethreshold", "integer", 4000, "Connections before idle ones are closed"),
    ("ipc_client_kill_max", "ipc.client.kill.max", "integer", 10, "Idle connections closed at once"),
    ("ipc_client_tcpnodelay", "ipc.client.tcpnodelay", "boolean", True, "TCP_NODELAY on IPC clients"),
    ("ipc_server_tcpnodelay", "ipc.server.tcpnodelay", "boolean", True, "TCP_NODELAY on IPC servers"),
    ("ipc_server_listen_queue_size", "ipc.server.listen.queue.size", "integer", 128, "IPC server listen backlog"),
    ("ipc_maximum_data_length", "ipc.maximum.data.length", "integer", 67108864, "Largest IPC message"),
    ("hadoop_http_staticuser_user", "hadoop.http.staticuser.user", "string", "dr.who", "User of unauthenticated web UI requests"),
    ("hadoop_security_group_mapping", "hadoop.security.group.mapping", "string",
     "org.apache.hadoop.security.JniBasedUnixGroupsMappingWithFallback", "User to group mapping"),
    ("hadoop_security_groups_cache_secs", "hadoop.security.groups.cache.secs", "integer", 300, "Group mapping cache"),
    ("hadoop_rpc_protection", "hadoop.rpc.protection", "string", "authentication", "SASL RPC protection: authentication, integrity, privacy"),
    ("hadoop_security_token_service_use_ip", "hadoop.security.token.service.use_ip", "boolean", True, "Token services named by IP"),
]

CASSANDRA = [Knob(k, k, t, d, desc, "CASSANDRA_" + k.upper()) for k, t, d, desc in _C]
HDFS_SITE = [Knob(k, prop, t, d, desc, k.upper()) for k, prop, t, d, desc in _H]
CORE_SITE = [Knob(k, prop, t, d, desc, k.upper()) for k, prop, t, d, desc in _CORE]


# -- generation ------------------------------------------------------------------------------------
def _value(k: Knob) -> str:
    return ("true" if k.default else "false") if k.type == "boolean" else str(k.default)


def _guarded(k: Knob, line: str) -> str:
    """A knob whose default is empty only appears when it is set."""
    return f"{{{{#{k.env}}}}}{line}{{{{/{k.env}}}}}" if _value(k) == "" else line


def template_lines(knobs: List[Knob], fmt: str) -> List[str]:
    if fmt == "yaml":
        return [_guarded(k, f"{k.setting}: {{{{{k.env}}}}}") for k in knobs]
    return [_guarded(k, f"  <property><name>{k.setting}</name><value>{{{{{k.env}}}}}</value></property>")
            for k in knobs]


def env_lines(knobs: List[Knob], section: str) -> List[str]:
    return [f'    "TASKCFG_ALL_{k.env}": "{{{{{section}.{k.key}}}}}",' for k in knobs]


def option_schema(k: Knob) -> dict:
    return OrderedDict([("description", f"{k.description} ({k.setting})"), ("type", k.type),
                        ("default", k.default)])


BEGIN, END = "knobs:begin", "knobs:end"


def _replace_region(text: str, lines: List[str], comment: Tuple[str, str]) -> str:
    """Replaces the lines between the BEGIN and END marker lines (comments in the file's syntax)."""
    begin = f"{comment[0]} {BEGIN} (python -m dcos_commons_amd.tools.package_knobs){comment[1]}"
    end = f"{comment[0]} {END}{comment[1]}"
    pat = re.compile(r"^[ \t]*" + re.escape(comment[0]) + r" " + BEGIN + r".*?^[ \t]*" + re.escape(comment[0]) +
                     r" " + END + r"[^\n]*$", re.S | re.M)
    block = "\n".join([begin] + lines + [end])
    if not pat.search(text):
        raise ValueError("no generated region (markers) in file")
    return pat.sub(lambda m: block, text, count=1)


def _update_json_section(config: dict, section: str, knobs: List[Knob]) -> dict:
    props = config["properties"][section]["properties"]
    for k in knobs:
        props[k.key] = option_schema(k)
    return config


PACKAGES = {
    # framework: [(section, knobs, template file, template format)]
    "cassandra": [("cassandra", CASSANDRA, "cassandra.yaml", "yaml")],
    "hdfs": [("hdfs", HDFS_SITE, "hdfs-site.xml", "xml"), ("hdfs", CORE_SITE, "core-site.xml", "xml")],
}
_COMMENTS = {"yaml": ("#", ""), "xml": ("<!--", " -->")}


def render_files(framework: str, base: str = ROOT) -> Dict[str, str]:
    """Path -> the file's content with every generated region filled from the tables."""
    fw = os.path.join(base, "frameworks", framework)
    out: Dict[str, str] = {}
    cfg_path = os.path.join(fw, "universe", "config.json")
    mar_path = os.path.join(fw, "universe", "marathon.json.mustache")
    with open(cfg_path, encoding="utf-8") as f:
        config = json.load(f, object_pairs_hook=OrderedDict)
    with open(mar_path, encoding="utf-8") as f:
        marathon = f.read()
    envs: List[str] = []
    for section, knobs, tpl, fmt in PACKAGES[framework]:
        config = _update_json_section(config, section, knobs)
        envs.extend(env_lines(knobs, section))
        path = os.path.join(fw, "specs", tpl)
        if path in out:
            text = out[path]
        else:
            with open(path, encoding="utf-8") as f:
                text = f.read()
        out[path] = _replace_region(text, template_lines(knobs, fmt), _COMMENTS[fmt])
    out[cfg_path] = json.dumps(config, indent=2) + "\n"
    out[mar_path] = _replace_region(marathon, envs, ("{{!", "}}"))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--check", action="store_true", help="only report files that are out of date")
    args = ap.parse_args(argv)
    stale = []
    for framework in PACKAGES:
        for path, content in render_files(framework).items():
            with open(path, encoding="utf-8") as f:
                current = f.read()
            if current != content:
                stale.append(path)
                if not args.check:
                    with open(path, "w", encoding="utf-8") as f:
                        f.write(content)
    if args.check and stale:
        print("out of date: " + ", ".join(os.path.relpath(p, ROOT) for p in stale))
        return 1
    print(("rewrote " if stale and not args.check else "up to date: ") + ", ".join(
        os.path.relpath(p, ROOT) for p in stale) if stale else "all package knob regions up to date")
    return 0


if __name__ == "__main__":
    sys.exit(main())
