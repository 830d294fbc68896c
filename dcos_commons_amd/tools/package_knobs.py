"""Application tuning knobs of the shipped cassandra and hdfs packages, one table each, and the
generator that keeps the package files in sync with the tables.

Each knob is one setting of the application's own configuration file -- a ``cassandra.yaml`` key
(Cassandra 3.11) or an ``hdfs-site.xml`` / ``core-site.xml`` property (Hadoop 2.x) -- with its type
and the application's default. From a table the generator writes, between marker lines:

* the package option (``universe/config.json``: ``cassandra.<key>``, or for hdfs the reference
  package's own option path -- ``name_node.<key>``, ``data_node.<key>``, ``hdfs.<key>`` -- with
  type, default and description),
* the scheduler environment entry that carries it to every task (``marathon.json.mustache``:
  ``"TASKCFG_ALL_<ENV>": "{{<option path>}}"``; the scheduler's TaskEnvRouter hands
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
    key: str                 # option key under the package section (cassandra) or full option path (hdfs)
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

# -- hdfs-site.xml / core-site.xml ------------------------------------------------------------------
# (option path, property, type, default, description[, env]). Option paths, types and defaults are
# those of the reference package's universe options (frameworks/hdfs/universe/config.json: the
# name_node / data_node / journal_node / hdfs sections; numbers there are strings, e.g. "0.999f"), so
# an options file written for it installs unchanged; properties the reference does not expose keep
# an ``hdfs.`` path with the Hadoop 2.x default. The env defaults to _hadoop_env(path); an explicit
# one keeps the name an earlier release of this package used.
_H = [
    ("name_node.safemode_threshold-pct", "dfs.namenode.safemode.threshold-pct", "string",
     "0.999f", "Fraction of blocks reported before safe mode ends"),
    ("name_node.safemode_extension", "dfs.namenode.safemode.extension", "string",
     "30000", "Safe mode extension after the threshold (ms)"),
    ("name_node.safemode_min_datanodes", "dfs.namenode.safemode.min.datanodes", "string",
     "0", "DataNodes required before safe mode ends"),
    ("name_node.heartbeat_recheck_interval", "dfs.namenode.heartbeat.recheck-interval", "string",
     "60000", "Dead DataNode detection interval (ms)"),
    ("name_node.checkpoint_period", "dfs.namenode.checkpoint.period", "string", "3600", "Seconds between checkpoints"),
    ("name_node.checkpoint_txns", "dfs.namenode.checkpoint.txns", "string",
     "1000000", "Transactions between checkpoints"),
    ("name_node.checkpoint_check_period", "dfs.namenode.checkpoint.check.period", "string",
     "60", "Checkpoint trigger polling (s)"),
    ("name_node.num_checkpoints_retained", "dfs.namenode.num.checkpoints.retained", "string",
     "2", "Image checkpoints kept"),
    ("name_node.num_extra_edits_retained", "dfs.namenode.num.extra.edits.retained", "string",
     "1000000", "Extra edit transactions kept"),
    ("name_node.max_extra_edits_segments_retained", "dfs.namenode.max.extra.edits.segments.retained", "string",
     "10000", "Extra edit log segments kept"),
    ("name_node.replication_min", "dfs.namenode.replication.min", "string", "1", "Minimal block replication"),
    ("name_node.max_objects", "dfs.namenode.max.objects", "string", "0", "Files + directories + blocks cap (0: none)"),
    ("name_node.decommission_interval", "dfs.namenode.decommission.interval", "string",
     "30", "Decommission progress check (s)"),
    ("name_node.decommission_blocks_per_interval", "dfs.namenode.decommission.blocks.per.interval", "string",
     "500000", "Blocks checked per decommission interval"),
    ("name_node.replication_interval", "dfs.namenode.replication.interval", "string",
     "3", "Replication work computation period (s)"),
    ("name_node.accesstime_precision", "dfs.namenode.accesstime.precision", "string",
     "3600000", "Access time precision (ms; 0 disables)"),
    ("name_node.fs-limits_max-component-length", "dfs.namenode.fs-limits.max-component-length", "string",
     "255", "Longest path component"),
    ("name_node.fs-limits_max-directory-items", "dfs.namenode.fs-limits.max-directory-items", "string",
     "1048576", "Most items in one directory"),
    ("name_node.fs-limits_min-block-size", "dfs.namenode.fs-limits.min-block-size", "string",
     "1048576", "Smallest block size"),
    ("name_node.fs-limits_max-blocks-per-file", "dfs.namenode.fs-limits.max-blocks-per-file", "string",
     "1048576", "Most blocks in one file"),
    ("name_node.stale_datanode_interval", "dfs.namenode.stale.datanode.interval", "string",
     "30000", "DataNode considered stale after (ms)"),
    ("name_node.avoid_read_stale_datanode", "dfs.namenode.avoid.read.stale.datanode", "boolean",
     False, "Read from stale DataNodes last"),
    ("name_node.avoid_write_stale_datanode", "dfs.namenode.avoid.write.stale.datanode", "boolean",
     False, "Avoid writing to stale DataNodes"),
    ("name_node.write_stale_datanode_ratio", "dfs.namenode.write.stale.datanode.ratio", "string",
     "0.5f", "Stale fraction above which writes use them again"),
    ("name_node.invalidate_work_pct_per_iteration", "dfs.namenode.invalidate.work.pct.per.iteration", "string",
     "0.32f", "Invalidation work per heartbeat"),
    ("name_node.replication_work_multiplier_per_iteration", "dfs.namenode.replication.work.multiplier.per.iteration", "string",
     "2", "Replication work per heartbeat"),
    ("name_node.enable_retrycache", "dfs.namenode.enable.retrycache", "boolean",
     True, "Retry cache for non-idempotent RPCs"),
    ("name_node.retrycache_expirytime_millis", "dfs.namenode.retrycache.expirytime.millis", "string",
     "600000", "Retry cache entry lifetime"),
    ("name_node.retrycache_heap_percent", "dfs.namenode.retrycache.heap.percent", "string",
     "0.03f", "Heap share of the retry cache"),
    ("name_node.list_cache_pools_num_responses", "dfs.namenode.list.cache.pools.num.responses", "string",
     "100", "Cache pools per listing"),
    ("name_node.list_cache_directives_num_responses", "dfs.namenode.list.cache.directives.num.responses", "string",
     "100", "Cache directives per listing"),
    ("name_node.path_based_cache_refresh_interval_ms", "dfs.namenode.path.based.cache.refresh.interval.ms", "string",
     "30000", "Cache directive rescan interval"),
    ("name_node.edit_log_autoroll_multiplier_threshold", "dfs.namenode.edit.log.autoroll.multiplier.threshold", "string",
     "2.0", "Edit log roll threshold (x checkpoint txns)"),
    ("name_node.edit_log_autoroll_check_interval_ms", "dfs.namenode.edit.log.autoroll.check.interval.ms", "string",
     "300000", "Edit log roll check interval"),
    ("name_node.delegation_key_update-interval", "dfs.namenode.delegation.key.update-interval", "string",
     "86400000", "Delegation key update interval"),
    ("name_node.delegation_token_max-lifetime", "dfs.namenode.delegation.token.max-lifetime", "string",
     "604800000", "Delegation token lifetime"),
    ("name_node.delegation_token_renew-interval", "dfs.namenode.delegation.token.renew-interval", "string",
     "86400000", "Delegation token renewal interval"),
    ("name_node.inotify_max_events_per_rpc", "dfs.namenode.inotify.max.events.per.rpc", "string",
     "1000", "inotify events per RPC"),
    ("name_node.reject-unresolved-dn-topology-mapping", "dfs.namenode.reject-unresolved-dn-topology-mapping", "boolean",
     False, "Reject DataNodes without a topology mapping"),
    ("name_node.resource_check_interval", "dfs.namenode.resource.check.interval", "string",
     "5000", "Local storage check interval (ms)"),
    ("name_node.resource_du_reserved", "dfs.namenode.resource.du.reserved", "string",
     "104857600", "Space kept free on NameNode volumes"),
    ("name_node.resource_checked_volumes_minimum", "dfs.namenode.resource.checked.volumes.minimum", "string",
     "1", "Volumes that must have space"),
    ("name_node.startup_delay_block_deletion_sec", "dfs.namenode.startup.delay.block.deletion.sec", "string",
     "0", "Delay block deletion after start-up"),
    ("name_node.acls_enabled", "dfs.namenode.acls.enabled", "boolean", False, "POSIX ACLs"),
    ("name_node.xattrs_enabled", "dfs.namenode.xattrs.enabled", "boolean", True, "Extended attributes"),
    ("name_node.fs-limits_max-attrs-per-inode", "dfs.namenode.fs-limits.max-xattrs-per-inode", "string",
     "32", "Extended attributes per inode", "NAME_NODE_FS_LIMITS_MAX_XATTRS_PER_INODE"),
    ("name_node.fs-limits_max-attrs-size", "dfs.namenode.fs-limits.max-xattr-size", "string",
     "16384", "Largest extended attribute", "NAME_NODE_FS_LIMITS_MAX_XATTR_SIZE"),
    ("name_node.replication_considerLoad", "dfs.namenode.replication.considerLoad", "boolean",
     True, "Consider DataNode load when placing replicas", "NAME_NODE_REPLICATION_CONSIDER_LOAD"),
    ("name_node.logging_level", "dfs.namenode.logging.level", "string", "info", "NameNode: logging level"),
    ("name_node.name_dir_restore", "dfs.namenode.name.dir.restore", "boolean", False, "NameNode: name dir restore"),
    ("name_node.lazypersist_file_scrub_interval_sec", "dfs.namenode.lazypersist.file.scrub.interval.sec", "string",
     "300", "NameNode: lazypersist file scrub interval sec"),
    ("name_node.handler_count", "dfs.namenode.handler.count", "string", "10", "NameNode: handler count"),
    ("name_node.resource_checked_volumes", "dfs.namenode.resource.checked.volumes", "string",
     "", "NameNode: resource checked volumes"),
    ("name_node.plugins", "dfs.namenode.plugins", "string", "", "NameNode: plugins"),
    ("name_node.checkpoint_max-retries", "dfs.namenode.checkpoint.max-retries", "string",
     "3", "NameNode: checkpoint max retries"),
    ("name_node.support_allow_format", "dfs.namenode.support.allow.format", "boolean",
     True, "NameNode: support allow format"),
    ("name_node.audit_loggers", "dfs.namenode.audit.loggers", "string", "default", "NameNode: audit loggers"),
    ("name_node.edits_noeditlogchannelflush", "dfs.namenode.edits.noeditlogchannelflush", "boolean",
     False, "NameNode: edits noeditlogchannelflush"),
    ("name_node.path_based_cache_block_map_allocation_percent", "dfs.namenode.path.based.cache.block.map.allocation.percent", "string",
     "0.25", "NameNode: path based cache block map allocation percent"),
    ("name_node.path_based_cache_retry_interval_ms", "dfs.namenode.path.based.cache.retry.interval.ms", "string",
     "30000", "NameNode: path based cache retry interval ms"),
    ("name_node.list_encryption_zones_num_responses", "dfs.namenode.list.encryption.zones.num.responses", "string",
     "100", "NameNode: list encryption zones num responses"),
    ("name_node.legacy-oiv-image_dir", "dfs.namenode.legacy-oiv-image.dir", "string",
     "", "NameNode: legacy oiv image dir"),
    ("data_node.handler_count", "dfs.datanode.handler.count", "string", "10", "DataNode RPC handlers"),
    ("data_node.max_transfer_threads", "dfs.datanode.max.transfer.threads", "string",
     "4096", "DataNode transfer threads"),
    ("data_node.balance_bandwidthPerSec", "dfs.datanode.balance.bandwidthPerSec", "string",
     "1048576", "Balancer bandwidth per DataNode", "DATA_NODE_BALANCE_BANDWIDTH_PER_SEC"),
    ("data_node.du_reserved", "dfs.datanode.du.reserved", "string", "0", "Space kept free per DataNode volume"),
    ("data_node.failed_volumes_tolerated", "dfs.datanode.failed.volumes.tolerated", "string",
     "0", "Failed volumes before the DataNode stops"),
    ("data_node.directoryscan_interval", "dfs.datanode.directoryscan.interval", "string",
     "21600", "Directory scan interval (s)"),
    ("data_node.directoryscan_threads", "dfs.datanode.directoryscan.threads", "string", "1", "Directory scan threads"),
    ("data_node.readahead_bytes", "dfs.datanode.readahead.bytes", "string", "4193404", "Read-ahead"),
    ("data_node.drop_cache_behind_reads", "dfs.datanode.drop.cache.behind.reads", "boolean",
     False, "Drop page cache behind reads"),
    ("data_node.drop_cache_behind_writes", "dfs.datanode.drop.cache.behind.writes", "boolean",
     False, "Drop page cache behind writes"),
    ("data_node.sync_behind_writes", "dfs.datanode.sync.behind.writes", "boolean", False, "Sync behind writes"),
    ("data_node.use_datanode_hostname", "dfs.datanode.use.datanode.hostname", "boolean",
     False, "DataNodes connect to each other by hostname"),
    ("data_node.cache_revocation_timeout_ms", "dfs.datanode.cache.revocation.timeout.ms", "string",
     "900000", "Cache revocation timeout"),
    ("data_node.cache_revocation_polling_ms", "dfs.datanode.cache.revocation.polling.ms", "string",
     "500", "Cache revocation polling"),
    ("data_node.max_locked_memory", "dfs.datanode.max.locked.memory", "string",
     "0", "Memory for the DataNode's block cache"),
    ("data_node.slow_io_warning_threshold_ms", "dfs.datanode.slow.io.warning.threshold.ms", "string",
     "300", "Slow I/O warning threshold"),
    ("data_node.fsdatasetcache_max_threads_per_volume", "dfs.datanode.fsdatasetcache.max.threads.per.volume", "string",
     "4", "Cache threads per volume"),
    ("data_node.plugins", "dfs.datanode.plugins", "string", "", "DataNode: plugins"),
    ("data_node.shared_file_descriptor_paths", "dfs.datanode.shared.file.descriptor.paths", "string",
     "/dev/shm,/tmp", "DataNode: shared file descriptor paths"),
    ("data_node.hdfs-blocks-metadata_enabled", "dfs.datanode.hdfs-blocks-metadata.enabled", "boolean",
     False, "DataNode: hdfs blocks metadata enabled"),
    ("data_node.fsdataset_volume_choosing_policy", "dfs.datanode.fsdataset.volume.choosing.policy", "string",
     "org.apache.hadoop.hdfs.server.datanode.fsdataset.RoundRobinVolumeChoosingPolicy", "DataNode: fsdataset volume choosing policy"),
    ("data_node.available-space-volume-choosing-policy_balanced-space-threshold", "dfs.datanode.available-space-volume-choosing-policy.balanced-space-threshold", "string",
     "10737418240", "DataNode: available space volume choosing policy balanced space threshold"),
    ("data_node.available-space-volume-choosing-policy_balanced-space-preference-fraction", "dfs.datanode.available-space-volume-choosing-policy.balanced-space-preference-fraction", "string",
     "0.75f", "DataNode: available space volume choosing policy balanced space preference fraction"),
    ("data_node.block_id_layout_upgrade_threads", "dfs.datanode.block.id.layout.upgrade.threads", "string",
     "12", "DataNode: block id layout upgrade threads"),
    ("hdfs.name_node_service_handler_count", "dfs.namenode.service.handler.count", "integer",
     10, "NameNode service RPC handlers"),
    ("hdfs.heartbeat_interval", "dfs.heartbeat.interval", "string", "3", "DataNode heartbeat interval (s)"),
    ("hdfs.replication_max", "dfs.replication.max", "string", "512", "Maximal block replication"),
    ("hdfs.name_node_top_enabled", "dfs.namenode.top.enabled", "boolean", True, "Top users metrics"),
    ("hdfs.name_node_top_window_num_buckets", "dfs.namenode.top.window.num.buckets", "integer",
     10, "Top users window buckets"),
    ("hdfs.name_node_top_num_users", "dfs.namenode.top.num.users", "integer", 10, "Top users reported"),
    ("hdfs.name_node_audit_log_async", "dfs.namenode.audit.log.async", "boolean", False, "Asynchronous audit log"),
    ("hdfs.name_node_datanode_registration_ip_hostname_check", "dfs.namenode.datanode.registration.ip-hostname-check", "boolean",
     False, "Require resolvable DataNode addresses"),
    ("hdfs.name_node_lifeline_handler_ratio", "dfs.namenode.lifeline.handler.ratio", "number",
     0.1, "Lifeline RPC handler share"),
    ("hdfs.name_node_quota_init_threads", "dfs.namenode.quota.init-threads", "integer",
     4, "Quota initialisation threads"),
    ("hdfs.name_node_name_cache_threshold", "dfs.namenode.name.cache.threshold", "integer", 10, "Name cache threshold"),
    ("hdfs.name_node_blocks_per_postponedblocks_rescan", "dfs.namenode.blocks.per.postponedblocks.rescan", "integer",
     10000, "Postponed blocks rescanned per iteration"),
    ("hdfs.name_node_fslock_fair", "dfs.namenode.fslock.fair", "boolean", True, "Fair namesystem lock"),
    ("hdfs.name_node_write_lock_reporting_threshold_ms", "dfs.namenode.write-lock-reporting-threshold-ms", "integer",
     5000, "Long write lock holds are logged"),
    ("hdfs.name_node_read_lock_reporting_threshold_ms", "dfs.namenode.read-lock-reporting-threshold-ms", "integer",
     5000, "Long read lock holds are logged"),
    ("hdfs.name_node_max_full_block_report_leases", "dfs.namenode.max.full.block.report.leases", "integer",
     6, "Concurrent full block reports"),
    ("hdfs.name_node_full_block_report_lease_length_ms", "dfs.namenode.full.block.report.lease.length.ms", "integer",
     300000, "Full block report lease"),
    ("hdfs.ha_tail-edits_period", "dfs.ha.tail-edits.period", "string", "60", "Standby edit tailing period (s)"),
    ("hdfs.ha_log-roll_period", "dfs.ha.log-roll.period", "string", "120", "Active edit log roll period (s)"),
    ("hdfs.ha_zkfc_nn_http_timeout_ms", "dfs.ha.zkfc.nn.http.timeout.ms", "integer",
     20000, "ZKFC health check HTTP timeout"),
    ("hdfs.ha_standby_checkpoints", "dfs.ha.standby.checkpoints", "boolean", True, "The standby NameNode checkpoints"),
    ("hdfs.image_compression_codec", "dfs.image.compression.codec", "string",
     "org.apache.hadoop.io.compress.SnappyCodec", "fsimage compression codec"),
    ("hdfs.image_transfer_timeout", "dfs.image.transfer.timeout", "string", "60000", "fsimage transfer timeout"),
    ("hdfs.image_transfer_bandwidthPerSec", "dfs.image.transfer.bandwidthPerSec", "string",
     "0", "fsimage transfer throttle (0: none)", "IMAGE_TRANSFER_BANDWIDTH_PER_SEC"),
    ("hdfs.image_transfer_chunksize", "dfs.image.transfer.chunksize", "string", "65536", "fsimage transfer chunk size"),
    ("hdfs.blocksize", "dfs.blocksize", "string", "134217728", "Default block size of new files"),
    ("hdfs.block_scanner_volume_bytes_per_second", "dfs.block.scanner.volume.bytes.per.second", "integer",
     1048576, "Block scanner throttle per volume"),
    ("hdfs.bytes-per-checksum", "dfs.bytes-per-checksum", "string", "512", "Bytes per checksum"),
    ("hdfs.checksum_type", "dfs.checksum.type", "string", "CRC32C", "Checksum type"),
    ("hdfs.client-write-packet-size", "dfs.client-write-packet-size", "string", "65536", "Client write packet size"),
    ("hdfs.client_block_write_retries", "dfs.client.block.write.retries", "string", "3", "Block write retries"),
    ("hdfs.client_block_write_replace-datanode-on-failure_enable", "dfs.client.block.write.replace-datanode-on-failure.enable", "boolean",
     True, "Replace failed DataNodes in a write pipeline"),
    ("hdfs.client_block_write_replace-datanode-on-failure_policy", "dfs.client.block.write.replace-datanode-on-failure.policy", "string",
     "DEFAULT", "Pipeline DataNode replacement policy"),
    ("hdfs.client_block_write_replace-datanode-on-failure_best-effort", "dfs.client.block.write.replace-datanode-on-failure.best-effort", "boolean",
     False, "Continue when no replacement DataNode is found"),
    ("hdfs.client_read_shortcircuit", "dfs.client.read.shortcircuit", "boolean",
     True, "Short-circuit local reads (needs dfs.domain.socket.path)"),
    ("hdfs.client_read_shortcircuit_streams_cache_size", "dfs.client.read.shortcircuit.streams.cache.size", "string",
     "256", "Short-circuit file descriptor cache size"),
    ("hdfs.client_read_shortcircuit_streams_cache_expiry_ms", "dfs.client.read.shortcircuit.streams.cache.expiry.ms", "string",
     "300000", "Short-circuit file descriptor cache expiry"),
    ("hdfs.client_socket_timeout", "dfs.client.socket-timeout", "integer", 60000, "Client socket timeout"),
    ("hdfs.client_failover_max_attempts", "dfs.client.failover.max.attempts", "string",
     "15", "Client failover attempts"),
    ("hdfs.client_failover_sleep_base_millis", "dfs.client.failover.sleep.base.millis", "string",
     "500", "Client failover backoff base"),
    ("hdfs.client_failover_sleep_max_millis", "dfs.client.failover.sleep.max.millis", "string",
     "15000", "Client failover backoff cap"),
    ("hdfs.client_retry_policy_enabled", "dfs.client.retry.policy.enabled", "boolean",
     False, "Client RPC retry policy"),
    ("hdfs.client_use_datanode_hostname", "dfs.client.use.datanode.hostname", "boolean",
     False, "Clients connect to DataNodes by hostname"),
    ("hdfs.client_context", "dfs.client.context", "string", "default", "Client cache context name"),
    ("hdfs.client_mmap_enabled", "dfs.client.mmap.enabled", "boolean", True, "Zero-copy reads through mmap"),
    ("hdfs.client_mmap_cache_size", "dfs.client.mmap.cache.size", "string", "256", "mmap regions cached"),
    ("hdfs.client_mmap_cache_timeout_ms", "dfs.client.mmap.cache.timeout.ms", "string", "3600000", "mmap cache expiry"),
    ("hdfs.client_short_circuit_replica_stale_threshold_ms", "dfs.client.short.circuit.replica.stale.threshold.ms", "string",
     "1800000", "Short-circuit replica staleness"),
    ("hdfs.data_node_balance_max_concurrent_moves", "dfs.datanode.balance.max.concurrent.moves", "integer",
     5, "Concurrent balancer moves"),
    ("hdfs.data_node_scan_period_hours", "dfs.datanode.scan.period.hours", "integer", 504, "Block scanner period"),
    ("hdfs.data_node_socket_write_timeout", "dfs.datanode.socket.write.timeout", "integer",
     480000, "DataNode socket write timeout"),
    ("hdfs.data_node_block_pinning_enabled", "dfs.datanode.block-pinning.enabled", "boolean", False, "Block pinning"),
    ("hdfs.data_node_bp_ready_timeout", "dfs.datanode.bp-ready.timeout", "integer", 20, "Block pool ready timeout (s)"),
    ("hdfs.data_node_cached_dfsused_check_interval_ms", "dfs.datanode.cached-dfsused.check.interval.ms", "integer",
     600000, "Cached dfsUsed validity"),
    ("hdfs.data_node_transfer_socket_send_buffer_size", "dfs.datanode.transfer.socket.send.buffer.size", "integer",
     131072, "Transfer socket send buffer"),
    ("hdfs.data_node_transfer_socket_recv_buffer_size", "dfs.datanode.transfer.socket.recv.buffer.size", "integer",
     131072, "Transfer socket receive buffer"),
    ("hdfs.data_node_lazywriter_interval_sec", "dfs.datanode.lazywriter.interval.sec", "integer",
     60, "Lazy persist writer interval"),
    ("hdfs.qjournal_start_segment_timeout_ms", "dfs.qjournal.start-segment.timeout.ms", "integer",
     20000, "Quorum journal start-segment timeout"),
    ("hdfs.qjournal_prepare_recovery_timeout_ms", "dfs.qjournal.prepare-recovery.timeout.ms", "integer",
     120000, "Quorum journal prepare-recovery timeout"),
    ("hdfs.qjournal_accept_recovery_timeout_ms", "dfs.qjournal.accept-recovery.timeout.ms", "integer",
     120000, "Quorum journal accept-recovery timeout"),
    ("hdfs.qjournal_finalize_segment_timeout_ms", "dfs.qjournal.finalize-segment.timeout.ms", "integer",
     120000, "Quorum journal finalize-segment timeout"),
    ("hdfs.qjournal_select_input_streams_timeout_ms", "dfs.qjournal.select-input-streams.timeout.ms", "integer",
     20000, "Quorum journal select-input-streams timeout"),
    ("hdfs.qjournal_get_journal_state_timeout_ms", "dfs.qjournal.get-journal-state.timeout.ms", "integer",
     120000, "Quorum journal get-state timeout"),
    ("hdfs.qjournal_new_epoch_timeout_ms", "dfs.qjournal.new-epoch.timeout.ms", "integer",
     120000, "Quorum journal new-epoch timeout"),
    ("hdfs.qjournal_write_txns_timeout_ms", "dfs.qjournal.write-txns.timeout.ms", "integer",
     20000, "Quorum journal write timeout"),
    ("hdfs.qjournal_queued_edits_limit_mb", "dfs.qjournal.queued-edits.limit.mb", "integer",
     10, "Queued edits per JournalNode"),
    ("hdfs.encrypt_data_transfer", "dfs.encrypt.data.transfer", "boolean", False, "Encrypt block data transfer"),
    ("hdfs.encrypt_data_transfer_algorithm", "dfs.encrypt.data.transfer.algorithm", "string",
     "", "Data transfer encryption algorithm (3des, rc4)"),
    ("hdfs.encrypt_data_transfer_cipher_key_bitlength", "dfs.encrypt.data.transfer.cipher.key.bitlength", "string",
     "128", "Data transfer cipher key length"),
    ("hdfs.encrypt_data_transfer_cipher_suites", "dfs.encrypt.data.transfer.cipher.suites", "string",
     "", "Data transfer cipher suites (AES/CTR/NoPadding)"),
    ("hdfs.data_transfer_protection", "dfs.data.transfer.protection", "string",
     "", "SASL data transfer protection: authentication, integrity, privacy"),
    ("hdfs.permissions_superusergroup", "dfs.permissions.superusergroup", "string", "supergroup", "Super-user group"),
    ("hdfs.administrators", "dfs.cluster.administrators", "string",
     "core,centos,azureuser,hdfs,nobody", "ACL of cluster administrators", "CLUSTER_ADMINISTRATORS"),
    ("hdfs.webhdfs_enabled", "dfs.webhdfs.enabled", "boolean", True, "WebHDFS REST API"),
    ("hdfs.webhdfs_rest_csrf_enabled", "dfs.webhdfs.rest-csrf.enabled", "boolean", False, "WebHDFS CSRF protection"),
    ("hdfs.webhdfs_ugi_expire_after_access", "dfs.webhdfs.ugi.expire.after.access", "integer",
     600000, "WebHDFS UGI cache expiry"),
    ("hdfs.user_home_dir_prefix", "dfs.user.home.dir.prefix", "string", "/user", "Home directory prefix"),
    ("hdfs.storage_policy_enabled", "dfs.storage.policy.enabled", "boolean", True, "Storage policies"),
    ("hdfs.stream-buffer-size", "dfs.stream-buffer-size", "string", "4096", "Stream buffer size"),
    ("hdfs.domain_socket_path", "dfs.domain.socket.path", "string", "", "UNIX domain socket for short-circuit reads"),
    ("hdfs.block_access_key_update_interval", "dfs.block.access.key.update.interval", "string",
     "600", "Block access key update interval (min)"),
    ("hdfs.block_access_token_lifetime", "dfs.block.access.token.lifetime", "string",
     "600", "Block access token lifetime (min)"),
    ("hdfs.default_chunk_view_size", "dfs.default.chunk.view.size", "string", "32768", "Bytes shown in the browser"),
    ("hdfs.blockreport_intervalMsec", "dfs.blockreport.intervalMsec", "string",
     "21600000", "Full block report interval", "BLOCKREPORT_INTERVAL_MSEC"),
    ("hdfs.blockreport_initialDelay", "dfs.blockreport.initialDelay", "string",
     "0", "First block report delay (s)", "BLOCKREPORT_INITIAL_DELAY"),
    ("hdfs.blockreport_split_threshold", "dfs.blockreport.split.threshold", "string",
     "1000000", "Blocks above which reports are split per volume"),
    ("hdfs.cachereport_intervalmsec", "dfs.cachereport.intervalMsec", "string",
     "10000", "Cache report interval", "CACHEREPORT_INTERVAL_MSEC"),
    ("hdfs.block_misreplication_processing_limit", "dfs.block.misreplication.processing.limit", "integer",
     10000, "Mis-replicated blocks processed per run"),
    ("hdfs.block_replicator_classname", "dfs.block.replicator.classname", "string",
     "org.apache.hadoop.hdfs.server.blockmanagement.BlockPlacementPolicyDefault", "Block placement policy"),
    ("hdfs.xframe_enabled", "dfs.xframe.enabled", "boolean", True, "X-Frame-Options header on the web UIs"),
    ("hdfs.xframe_value", "dfs.xframe.value", "string", "SAMEORIGIN", "X-Frame-Options value"),
    ("hdfs.http_client_retry_policy_enabled", "dfs.http.client.retry.policy.enabled", "boolean",
     False, "WebHDFS client retry policy"),
    ("hdfs.client_https_need_auth", "dfs.client.https.need-auth", "boolean",
     False, "Require client certificates on HTTPS"),
    ("hdfs.compress_image", "dfs.image.compress", "boolean", True, "HDFS: image compress"),
    ("hdfs.hadoop_hdfs_configuration_version", "hadoop.hdfs.configuration.version", "string",
     "1", "Hadoop: hdfs configuration version"),
    ("hdfs.client_cached_conn_retry", "dfs.client.cached.conn.retry", "string", "3", "Client: cached conn retry"),
    ("hdfs.https_server_keystore_resource", "dfs.https.server.keystore.resource", "string",
     "ssl-server.xml", "HDFS: https server keystore resource"),
    ("hdfs.client_https_keystore_resource", "dfs.client.https.keystore.resource", "string",
     "ssl-client.xml", "Client: https keystore resource"),
    ("hdfs.hosts", "dfs.hosts", "string", "", "HDFS: hosts"),
    ("hdfs.hosts_exclude", "dfs.hosts.exclude", "string", "", "HDFS: hosts exclude"),
    ("hdfs.client_write_exclude_nodes_cache_expiry_interval_millis", "dfs.client.write.exclude.nodes.cache.expiry.interval.millis", "string",
     "600000", "Client: write exclude nodes cache expiry interval millis"),
    ("hdfs.client_failover_connection_retries", "dfs.client.failover.connection.retries", "string",
     "0", "Client: failover connection retries"),
    ("hdfs.client_failover_connection_retries_on_timeouts", "dfs.client.failover.connection.retries.on.timeouts", "string",
     "0", "Client: failover connection retries on timeouts"),
    ("hdfs.client_datanode-restart_timeout", "dfs.client.datanode-restart.timeout", "string",
     "30", "Client: datanode restart timeout"),
    ("hdfs.support_append", "dfs.support.append", "boolean", True, "HDFS: support append"),
    ("hdfs.client_local_interfaces", "dfs.client.local.interfaces", "string", "", "Client: local interfaces"),
    ("hdfs.short_circuit_shared_memory_watcher_interrupt_check_ms", "dfs.short.circuit.shared.memory.watcher.interrupt.check.ms", "string",
     "60000", "HDFS: short circuit shared memory watcher interrupt check ms"),
    ("hdfs.fuse_connection_timeout", "hadoop.fuse.connection.timeout", "string",
     "300", "Hadoop: fuse connection timeout"),
    ("hdfs.fuse_timer_period", "hadoop.fuse.timer.period", "string", "5", "Hadoop: fuse timer period"),
    ("hdfs.metrics_percentiles_intervals", "dfs.metrics.percentiles.intervals", "string",
     "", "HDFS: metrics percentiles intervals"),
    ("hdfs.trustedchannel_resolver_class", "dfs.trustedchannel.resolver.class", "string",
     "", "HDFS: trustedchannel resolver class"),
    ("hdfs.data_transfer_saslproperties_resolver_class", "dfs.data.transfer.saslproperties.resolver.class", "string",
     "", "HDFS: data transfer saslproperties resolver class"),
    ("hdfs.client_file-block-storage-locations_num-threads", "dfs.client.file-block-storage-locations.num-threads", "string",
     "10", "Client: file block storage locations num threads"),
    ("hdfs.client_file-block-storage-locations_timeout_millis", "dfs.client.file-block-storage-locations.timeout.millis", "string",
     "1000", "Client: file block storage locations timeout millis"),
    ("hdfs.client_cache_drop_behind_writes", "dfs.client.cache.drop.behind.writes", "string",
     "", "Client: cache drop behind writes"),
    ("hdfs.client_cache_drop_behind_reads", "dfs.client.cache.drop.behind.reads", "string",
     "", "Client: cache drop behind reads"),
    ("hdfs.client_cache_readahead", "dfs.client.cache.readahead", "string", "", "Client: cache readahead"),
    ("hdfs.client_mmap_retry_timeout_ms", "dfs.client.mmap.retry.timeout.ms", "string",
     "300000", "Client: mmap retry timeout ms"),
    ("hdfs.webhdfs_user_provider_user_pattern", "dfs.webhdfs.user.provider.user.pattern", "string",
     "^[A-Za-z_][A-Za-z0-9._-]*[$]?$", "HDFS: webhdfs user provider user pattern"),
    ("hdfs.ha_fencing_methods", "dfs.ha.fencing.methods", "string", "shell(/bin/true)", "HA: fencing methods"),
    ("hdfs.client_read_shortcircuit_skip_checksum", "dfs.client.read.shortcircuit.skip.checksum", "boolean",
     False, "Client: read shortcircuit skip checksum"),
    ("hdfs.block_local-path-access_user", "dfs.block.local-path-access.user", "string",
     "", "HDFS: block local path access user"),
    ("hdfs.client_domain_socket_data_traffic", "dfs.client.domain.socket.data.traffic", "boolean",
     False, "Client: domain socket data traffic"),
    ("hdfs.client_slow_io_warning_threshold_ms", "dfs.client.slow.io.warning.threshold.ms", "string",
     "30000", "Client: slow io warning threshold ms"),
    ("hdfs.encryption_key_provider_uri", "dfs.encryption.key.provider.uri", "string",
     "", "HDFS: encryption key provider uri"),
    ("hdfs.namenode_rpc-bind-host_name_node_0", "dfs.namenode.rpc-bind-host.hdfs.name-0-node", "string",
     "0.0.0.0", "NameNode: rpc bind host hdfs name 0 node"),
    ("hdfs.namenode_rpc-bind-host_name_node_1", "dfs.namenode.rpc-bind-host.hdfs.name-1-node", "string",
     "0.0.0.0", "NameNode: rpc bind host hdfs name 1 node"),
    ("hdfs.namenode_http-bind-host_name_node_0", "dfs.namenode.http-bind-host.hdfs.name-0-node", "string",
     "0.0.0.0", "NameNode: http bind host hdfs name 0 node"),
    ("hdfs.namenode_http-bind-host_name_node_1", "dfs.namenode.http-bind-host.hdfs.name-1-node", "string",
     "0.0.0.0", "NameNode: http bind host hdfs name 1 node"),
    ("hdfs.namenode_servicerpc_address_namenode_0", "dfs.namenode.servicerpc-address.hdfs.name-0-node", "string",
     "", "NameNode: servicerpc address hdfs name 0 node"),
    ("hdfs.namenode_servicerpc_address_namenode_1", "dfs.namenode.servicerpc-address.hdfs.name-1-node", "string",
     "", "NameNode: servicerpc address hdfs name 1 node"),
    ("hdfs.namenode_servicerpc_bind_host_namenode_0", "dfs.namenode.servicerpc-bind-host.hdfs.name-0-node", "string",
     "", "NameNode: servicerpc bind host hdfs name 0 node"),
    ("hdfs.namenode_servicerpc_bind_host_namenode_1", "dfs.namenode.servicerpc-bind-host.hdfs.name-1-node", "string",
     "", "NameNode: servicerpc bind host hdfs name 1 node"),
]

_CORE = [
    ("hdfs.io_file_buffer_size", "io.file.buffer.size", "string", "4096", "I/O buffer size"),
    ("hdfs.fs_trash_interval", "fs.trash.interval", "string",
     "0", "Minutes deleted files stay in the trash (0: no trash)"),
    ("hdfs.fs_trash_checkpoint_interval", "fs.trash.checkpoint.interval", "string",
     "0", "Minutes between trash checkpoints"),
    ("hdfs.fs_df_interval", "fs.df.interval", "string", "60000", "Disk usage statistics refresh"),
    ("hdfs.fs_du_interval", "fs.du.interval", "string", "600000", "Space used refresh"),
    ("hdfs.ipc_client_connect_max_retries", "ipc.client.connect.max.retries", "string",
     "300", "IPC connection retries"),
    ("hdfs.ipc_client_connect_retry_interval", "ipc.client.connect.retry.interval", "string",
     "1000", "IPC connection retry interval"),
    ("hdfs.ipc_client_connect_timeout", "ipc.client.connect.timeout", "string", "20000", "IPC connection timeout"),
    ("hdfs.ipc_client_connect_max_retries_on_timeouts", "ipc.client.connect.max.retries.on.timeouts", "string",
     "45", "IPC retries on connection timeouts"),
    ("hdfs.ipc_client_connection_maxidletime", "ipc.client.connection.maxidletime", "string",
     "10000", "Idle IPC connection lifetime"),
    ("hdfs.ipc_client_idlethreshold", "ipc.client.idlethreshold", "string",
     "4000", "Connections before idle ones are closed"),
    ("hdfs.ipc_client_kill_max", "ipc.client.kill.max", "string", "10", "Idle connections closed at once"),
    ("hdfs.ipc_client_tcpnodelay", "ipc.client.tcpnodelay", "boolean", True, "TCP_NODELAY on IPC clients"),
    ("hdfs.ipc_server_tcpnodelay", "ipc.server.tcpnodelay", "boolean", True, "TCP_NODELAY on IPC servers"),
    ("hdfs.ipc_server_listen_queue_size", "ipc.server.listen.queue.size", "string", "45", "IPC server listen backlog"),
    ("hdfs.ipc_maximum_data_length", "ipc.maximum.data.length", "string", "67108864", "Largest IPC message"),
    ("hdfs.hadoop_http_staticuser_user", "hadoop.http.staticuser.user", "string",
     "dr.who", "User of unauthenticated web UI requests"),
    ("hdfs.security_group_mapping", "hadoop.security.group.mapping", "string",
     "org.apache.hadoop.security.JniBasedUnixGroupsMappingWithFallback", "User to group mapping", "HADOOP_SECURITY_GROUP_MAPPING"),
    ("hdfs.security_groups_cache_secs", "hadoop.security.groups.cache.secs", "string",
     "300", "Group mapping cache", "HADOOP_SECURITY_GROUPS_CACHE_SECS"),
    ("hdfs.rpc_protection", "hadoop.rpc.protection", "string",
     "authentication", "SASL RPC protection: authentication, integrity, privacy", "HADOOP_RPC_PROTECTION"),
    ("hdfs.hadoop_security_token_service_use_ip", "hadoop.security.token.service.use_ip", "boolean",
     True, "Token services named by IP"),
    ("hdfs.common_configuration_version", "hadoop.common.configuration.version", "string",
     "0.23.0", "Hadoop: common configuration version"),
    ("hdfs.tmp_dir", "hadoop.tmp.dir", "string", "/tmp/hadoop-$(whoami)", "Hadoop: tmp dir"),
    ("hdfs.http_filter_initializer", "hadoop.http.filter.initializers", "string",
     "org.apache.hadoop.security.AuthenticationFilterInitializer", "HTTP: filter initializers"),
    ("hdfs.security_groups_negative-cache_secs", "hadoop.security.groups.negative-cache.secs", "string",
     "30", "Security: groups negative cache secs"),
    ("hdfs.security_groups_cache_warn_after_ms", "hadoop.security.groups.cache.warn.after.ms", "string",
     "5000", "Security: groups cache warn after ms"),
    ("hdfs.security_service_user_name_key", "hadoop.security.service.user.name.key", "string",
     "", "Security: service user name key"),
    ("hdfs.security_service_uid_cache_secs", "hadoop.security.uid.cache.secs", "string",
     "14400", "Security: uid cache secs"),
    ("hdfs.security_saslproperties_resolver_class", "hadoop.security.saslproperties.resolver.class", "string",
     "", "Security: saslproperties resolver class"),
    ("hdfs.work_around_non_threadsafe_getpwuid", "hadoop.work.around.non.threadsafe.getpwuid", "boolean",
     False, "Hadoop: work around non threadsafe getpwuid"),
    ("hdfs.kerberos_kinit_command", "hadoop.kerberos.kinit.command", "string",
     "kinit", "Hadoop: kerberos kinit command"),
    ("hdfs.hadoop_security_instrumentation_requires_admin", "hadoop.security.instrumentation.requires.admin", "boolean",
     False, "Security: instrumentation requires admin"),
    ("hdfs.io_bytes_per_checksum", "io.bytes.per.checksum", "string", "512", "I/O: bytes per checksum"),
    ("hdfs.io_skip_checksum_errors", "io.skip.checksum.errors", "boolean", False, "I/O: skip checksum errors"),
    ("hdfs.io_compression_codecs", "io.compression.codecs", "string", "", "I/O: compression codecs"),
    ("hdfs.io_compression_codec_bzip2_library", "io.compression.codec.bzip2.library", "string",
     "system-native", "I/O: compression codec bzip2 library"),
    ("hdfs.io_serializations", "io.serializations", "string",
     "org.apache.hadoop.io.serializer.WritableSerialization,org.apache.hadoop.io.serializer.avro.AvroSpecificSerialization,org.apache.hadoop.io.serializer.avro.AvroReflectSerialization", "I/O: serializations"),
    ("hdfs.io_seqfile_local_dir", "io.seqfile.local.dir", "string",
     "${hadoop.tmp.dir}/io/local", "SequenceFile: local dir"),
    ("hdfs.io_map_index_skip", "io.map.index.skip", "string", "0", "I/O: map index skip"),
    ("hdfs.io_map_index_interval", "io.map.index.interval", "string", "128", "I/O: map index interval"),
    ("hdfs.fs_abstractfilesystem_file_impl", "fs.AbstractFileSystem.file.impl", "string",
     "org.apache.hadoop.fs.local.LocalFs", "AbstractFileSystem: file impl"),
    ("hdfs.fs_abstractfilesystem_har_impl", "fs.AbstractFileSystem.har.impl", "string",
     "org.apache.hadoop.fs.HarFs", "AbstractFileSystem: har impl"),
    ("hdfs.fs_abstractfilesystem_hdfs_impl", "fs.AbstractFileSystem.hdfs.impl", "string",
     "org.apache.hadoop.fs.Hdfs", "AbstractFileSystem: hdfs impl"),
    ("hdfs.fs_abstractfilesystem_viewfs_impl", "fs.AbstractFileSystem.viewfs.impl", "string",
     "org.apache.hadoop.fs.viewfs.ViewFs", "AbstractFileSystem: viewfs impl"),
    ("hdfs.fs_ftp_host", "fs.ftp.host", "string", "0.0.0.0", "FileSystem: ftp host"),
    ("hdfs.fs_ftp_host_port", "fs.ftp.host.port", "string", "21", "FileSystem: ftp host port"),
    ("hdfs.fs_s3_block_size", "fs.s3.block.size", "string", "67108864", "S3: block size"),
    ("hdfs.fs_s3_buffer_dir", "fs.s3.buffer.dir", "string", "${hadoop.tmp.dir}/s3", "S3: buffer dir"),
    ("hdfs.fs_s3_maxretries", "fs.s3.maxRetries", "string", "4", "S3: max retries"),
    ("hdfs.fs_s3_sleep_time_seconds", "fs.s3.sleepTimeSeconds", "string", "10", "S3: sleep time seconds"),
    ("hdfs.sf_swift_impl", "fs.swift.impl", "string",
     "org.apache.hadoop.fs.swift.snative.SwiftNativeFileSystem", "FileSystem: swift impl"),
    ("hdfs.fs_automatic_close", "fs.automatic.close", "boolean", True, "FileSystem: automatic close"),
    ("hdfs.fs_s3n_block_size", "fs.s3n.block.size", "string", "67108864", "S3N: block size"),
    ("hdfs.fs_s3n_multipart_uploads_enabled", "fs.s3n.multipart.uploads.enabled", "boolean",
     False, "S3N: multipart uploads enabled"),
    ("hdfs.fs_s3n_multipart_uploads_block_size", "fs.s3n.multipart.uploads.block.size", "string",
     "67108864", "S3N: multipart uploads block size"),
    ("hdfs.fs_s3n_multipart_copy_block_size", "fs.s3n.multipart.copy.block.size", "string",
     "5368709120", "S3N: multipart copy block size"),
    ("hdfs.fs_s3n_server-side-encrpytion-algorithm", "fs.s3n.server-side-encryption-algorithm", "string",
     "", "S3N: server side encryption algorithm"),
    ("hdfs.fs_s3n_access_key", "fs.s3a.access.key", "string", "", "S3A: access key"),
    ("hdfs.fs_s3n_secret_key", "fs.s3a.secret.key", "string", "", "S3A: secret key"),
    ("hdfs.fs_s3n_connection_maximum", "fs.s3a.connection.maximum", "string", "15", "S3A: connection maximum"),
    ("hdfs.fs_s3n_connection_ssl_enabled", "fs.s3a.connection.ssl.enabled", "boolean",
     True, "S3A: connection ssl enabled"),
    ("hdfs.fs_s3n_attempts_maximum", "fs.s3a.attempts.maximum", "string", "10", "S3A: attempts maximum"),
    ("hdfs.fs_s3n_connection_timeout", "fs.s3a.connection.timeout", "string", "5000", "S3A: connection timeout"),
    ("hdfs.fs_s3n_paging_maximum", "fs.s3a.paging.maximum", "string", "5000", "S3A: paging maximum"),
    ("hdfs.fs_s3n_multipart_size", "fs.s3a.multipart.size", "string", "104857600", "S3A: multipart size"),
    ("hdfs.fs_s3n_multipart_threshold", "fs.s3a.multipart.threshold", "string",
     "2147483647", "S3A: multipart threshold"),
    ("hdfs.fs_s3n_acl_default", "fs.s3a.acl.default", "string", "", "S3A: acl default"),
    ("hdfs.fs_s3n_multipart_purge", "fs.s3a.multipart.purge", "boolean", False, "S3A: multipart purge"),
    ("hdfs.fs_s3n_multipart_purge_age", "fs.s3a.multipart.purge.age", "string", "86400", "S3A: multipart purge age"),
    ("hdfs.fs_s3n_buffer_dir", "fs.s3a.buffer.dir", "string", "${hadoop.tmp.dir}/s3a", "S3A: buffer dir"),
    ("hdfs.fs_s3n_impl", "fs.s3a.impl", "string", "org.apache.hadoop.fs.s3a.S3AFileSystem", "S3A: impl"),
    ("hdfs.io_seqfile_compress_blocksize", "io.seqfile.compress.blocksize", "string",
     "1000000", "SequenceFile: compress blocksize"),
    ("hdfs.io_seqfile_lazydecompress", "io.seqfile.lazydecompress", "boolean", True, "SequenceFile: lazydecompress"),
    ("hdfs.io_seqfile_sorter_recordlimit", "io.seqfile.sorter.recordlimit", "string",
     "1000000", "SequenceFile: sorter recordlimit"),
    ("hdfs.io_seqfile_bloom_size", "io.mapfile.bloom.size", "string", "1048576", "MapFile: bloom size"),
    ("hdfs.io_seqfile_bloom_error_rate", "io.mapfile.bloom.error.rate", "string", "0.005", "MapFile: bloom error rate"),
    ("hdfs.hadoop_util_hash_type", "hadoop.util.hash.type", "string", "murmur", "Hadoop: util hash type"),
    ("hdfs.hadoop_security_impersonation_provider_class", "hadoop.security.impersonation.provider.class", "string",
     "", "Security: impersonation provider class"),
    ("hdfs.hadoop_rpc_socket_factory_class_default", "hadoop.rpc.socket.factory.class.default", "string",
     "org.apache.hadoop.net.StandardSocketFactory", "RPC: socket factory class default"),
    ("hdfs.hadoop_rpc_socket_factory_class_client-protocol", "hadoop.rpc.socket.factory.class.ClientProtocol", "string",
     "", "RPC: socket factory class client protocol"),
    ("hdfs.hadoop_socks_server", "hadoop.socks.server", "string", "", "Hadoop: socks server"),
    ("hdfs.file_stream-buffer-size", "file.stream-buffer-size", "string", "4096", "file://: stream buffer size"),
    ("hdfs.file_bytes-per-checksum", "file.bytes-per-checksum", "string", "512", "file://: bytes per checksum"),
    ("hdfs.file_client-write-packet-size", "file.client-write-packet-size", "string",
     "65536", "file://: client write packet size"),
    ("hdfs.file_blocksize", "file.blocksize", "string", "67108864", "file://: blocksize"),
    ("hdfs.file_replication", "file.replication", "string", "1", "file://: replication"),
    ("hdfs.s3_stream-buffer-size", "s3.stream-buffer-size", "string", "4096", "s3://: stream buffer size"),
    ("hdfs.s3_bytes-per-checksum", "s3.bytes-per-checksum", "string", "512", "s3://: bytes per checksum"),
    ("hdfs.s3_client-write-packet-size", "s3.client-write-packet-size", "string",
     "65536", "s3://: client write packet size"),
    ("hdfs.s3_blocksize", "s3.blocksize", "string", "67108864", "s3://: blocksize"),
    ("hdfs.s3_replication", "s3.replication", "string", "3", "s3://: replication"),
    ("hdfs.s3native_stream-buffer-size", "s3native.stream-buffer-size", "string", "4096", "s3n://: stream buffer size"),
    ("hdfs.s3native_bytes-per-checksum", "s3native.bytes-per-checksum", "string", "512", "s3n://: bytes per checksum"),
    ("hdfs.s3native_client-write-packet-size", "s3native.client-write-packet-size", "string",
     "65536", "s3n://: client write packet size"),
    ("hdfs.s3native_blocksize", "s3native.blocksize", "string", "67108864", "s3n://: blocksize"),
    ("hdfs.s3native_replication", "s3native.replication", "string", "3", "s3n://: replication"),
    ("hdfs.ftp_stream-buffer-size", "ftp.stream-buffer-size", "string", "4096", "ftp://: stream buffer size"),
    ("hdfs.ftp_bytes-per-checksum", "ftp.bytes-per-checksum", "string", "512", "ftp://: bytes per checksum"),
    ("hdfs.ftp_client-write-packet-size", "ftp.client-write-packet-size", "string",
     "65536", "ftp://: client write packet size"),
    ("hdfs.ftp_blocksize", "ftp.blocksize", "string", "67108864", "ftp://: blocksize"),
    ("hdfs.ftp_replication", "ftp.replication", "string", "3", "ftp://: replication"),
    ("hdfs.tfile_io_chunk_size", "tfile.io.chunk.size", "string", "1048576", "TFile: io chunk size"),
    ("hdfs.tfile_io_output_buffer_size", "tfile.fs.output.buffer.size", "string",
     "262144", "TFile: fs output buffer size"),
    ("hdfs.tfile_fs_input_buffer_size", "tfile.fs.input.buffer.size", "string",
     "262144", "TFile: fs input buffer size"),
    ("hdfs.hadoop_http_authentication_token_validity", "hadoop.http.authentication.token.validity", "string",
     "36000", "HTTP: authentication token validity"),
    ("hdfs.hadoop_http_authentication_simple_anonymous_allowed", "hadoop.http.authentication.simple.anonymous.allowed", "boolean",
     True, "HTTP: authentication simple anonymous allowed"),
    ("hdfs.dfs_ha_fencing_ssh_connect-timeout", "dfs.ha.fencing.ssh.connect-timeout", "string",
     "30000", "HA: fencing ssh connect timeout"),
    ("hdfs.dfs_ha_fencing_ssh_private-key-files", "dfs.ha.fencing.ssh.private-key-files", "string",
     "", "HA: fencing ssh private key files"),
    ("hdfs.ha_zookeeper_session-timeout-ms", "ha.zookeeper.session-timeout.ms", "string",
     "5000", "HA: zookeeper session timeout ms"),
    ("hdfs.hadoop_ssl_keystores_factory_class", "hadoop.ssl.keystores.factory.class", "string",
     "org.apache.hadoop.security.ssl.FileBasedKeyStoresFactory", "SSL: keystores factory class"),
    ("hdfs.hadoop_ssl_require_client_cert", "hadoop.ssl.require.client.cert", "boolean",
     False, "SSL: require client cert"),
    ("hdfs.hadoop_jetty_logs_serve_aliases", "hadoop.jetty.logs.serve.aliases", "boolean",
     False, "Hadoop: jetty logs serve aliases"),
    ("hdfs.fs_permissions_umask-mode", "fs.permissions.umask-mode", "string",
     "022", "FileSystem: permissions umask mode"),
    ("hdfs.ha_health-monitor_connect-retry-interval_ms", "ha.health-monitor.connect-retry-interval.ms", "string",
     "1000", "HA: health monitor connect retry interval ms"),
    ("hdfs.ha_health-monitor_check-interval_ms", "ha.health-monitor.check-interval.ms", "string",
     "1000", "HA: health monitor check interval ms"),
    ("hdfs.ha_health-monitor_sleep-after-disconnect_ms", "ha.health-monitor.sleep-after-disconnect.ms", "string",
     "1000", "HA: health monitor sleep after disconnect ms"),
    ("hdfs.ha_health-monitor_rpc-timeout_ms", "ha.health-monitor.rpc-timeout.ms", "string",
     "45000", "HA: health monitor rpc timeout ms"),
    ("hdfs.ha_failover-controller_new-active_rpc-timeout_ms", "ha.failover-controller.new-active.rpc-timeout.ms", "string",
     "60000", "HA: failover controller new active rpc timeout ms"),
    ("hdfs.ha_failover-controller_graceful-fence_rpc-timeout_ms", "ha.failover-controller.graceful-fence.rpc-timeout.ms", "string",
     "5000", "HA: failover controller graceful fence rpc timeout ms"),
    ("hdfs.ha_failover-controller_graceful-fence_connection_retries", "ha.failover-controller.graceful-fence.connection.retries", "string",
     "1", "HA: failover controller graceful fence connection retries"),
    ("hdfs.ha_failover-controller_cli-check_rpc-timeout_ms", "ha.failover-controller.cli-check.rpc-timeout.ms", "string",
     "20000", "HA: failover controller cli check rpc timeout ms"),
    ("hdfs.ipc_client_fallback-to-simple-auth-allowed", "ipc.client.fallback-to-simple-auth-allowed", "boolean",
     False, "IPC: client fallback to simple auth allowed"),
    ("hdfs.fs_client_resolve_remote_symlinks", "fs.client.resolve.remote.symlinks", "boolean",
     True, "FileSystem: client resolve remote symlinks"),
    ("hdfs.nfs_exports_allowed_hosts", "nfs.exports.allowed.hosts", "string", "* rw", "NFS: exports allowed hosts"),
    ("hdfs.hadoop_user_group_static_mapping_overrides", "hadoop.user.group.static.mapping.overrides", "string",
     "", "Hadoop: user group static mapping overrides"),
    ("hdfs.rpc_metrics_quantile_enable", "rpc.metrics.quantile.enable", "boolean",
     False, "RPC: metrics quantile enable"),
    ("hdfs.rpc_metrics_percentiles_intervals", "rpc.metrics.percentiles.intervals", "string",
     "", "RPC: metrics percentiles intervals"),
    ("hdfs.hadoop_http_authentication_cookie_domain", "hadoop.http.authentication.cookie.domain", "string",
     "", "HTTP: authentication cookie domain"),
    ("hdfs.hadoop_http_authentication_kerberos_principal", "hadoop.http.authentication.kerberos.principal", "string",
     "HTTP/_HOST@LOCALHOST", "HTTP: authentication kerberos principal"),
    ("hdfs.hadoop_http_authentication_kerberos_keytab", "hadoop.http.authentication.kerberos.keytab", "string",
     "${user.home}/hadoop.keytab", "HTTP: authentication kerberos keytab"),
]

CASSANDRA = [Knob(k, k, t, d, desc, "CASSANDRA_" + k.upper()) for k, t, d, desc in _C]


def _hadoop_env(path: str) -> str:
    """``name_node.fs-limits_min-block-size`` -> ``NAME_NODE_FS_LIMITS_MIN_BLOCK_SIZE``; the ``hdfs``
    section adds no prefix."""
    section, key = path.split(".", 1)
    base = re.sub(r"[^A-Za-z0-9]", "_", key).upper()
    return base if section == "hdfs" else f"{section.upper()}_{base}"


HDFS_SITE = [Knob(path, prop, t, d, desc, env[0] if env else _hadoop_env(path)) for path, prop, t, d, desc, *env in _H]
CORE_SITE = [Knob(path, prop, t, d, desc, env[0] if env else _hadoop_env(path)) for path, prop, t, d, desc, *env in _CORE]


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


def _path(k: Knob, section: Optional[str]) -> str:
    """The option's path in config.json: ``<section>.<key>``, or the key itself when the table holds
    full paths (section None)."""
    return k.key if section is None else f"{section}.{k.key}"


def env_lines(knobs: List[Knob], section: Optional[str]) -> List[str]:
    return [f'    "TASKCFG_ALL_{k.env}": "{{{{{_path(k, section)}}}}}",' for k in knobs]


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


def _update_json_section(config: dict, section: Optional[str], knobs: List[Knob]) -> dict:
    for k in knobs:
        top, key = _path(k, section).split(".", 1)
        config["properties"][top]["properties"][key] = option_schema(k)
    return config


PACKAGES = {
    # framework: [(section (None: the knob keys are full option paths), knobs, template, format)]
    "cassandra": [("cassandra", CASSANDRA, "cassandra.yaml", "yaml")],
    "hdfs": [(None, HDFS_SITE, "hdfs-site.xml", "xml"), (None, CORE_SITE, "core-site.xml", "xml")],
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
