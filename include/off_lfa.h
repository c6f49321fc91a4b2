/*
 * off_lfa — provider-specific endpoint options of the offload-collective
 * provider libfabric_amd/liboff_lfa-fi.so (libfabric_amd/csrc/off_lfa.c).
 *
 * The provider registers under the name "off_lfa"; the "off_" prefix is what
 * makes libfabric's core class it as an offload provider
 * (src/fabric.c:508-510, include/ofi_util.h:1192-1202), and rxm then routes
 * every collective whose fi_query_collective succeeds to it when
 * FI_OFFLOAD_COLL_PROVIDER=off_lfa (rxm_fabric.c:131-139,
 * rxm_domain.c:878-893, rxm_ep.c:679-684).
 *
 * Options follow the provider-specific convention of include/rdma/fi_ext.h:
 * a 12-bit provider code shifted left 16 bits, negated.  Pass them to
 * fi_getopt / fi_setopt at level FI_OPT_ENDPOINT (0) on the off_lfa
 * endpoint.
 *
 * World bootstrap.  The first fi_join_collective with coll_addr ==
 * FI_ADDR_NOTAVAIL creates the RCCL communicator of the av_set's members
 * (rank = position of the owner endpoint's address in the set,
 * coll_coll.c:669-688).  Members agree on a 128-byte unique id exactly as
 * RCCL programs do: rank 0 reads one with fi_getopt(OFF_LFA_OPT_UNIQUE_ID),
 * the application ships it to the other members by any means, and every
 * member hands it in with fi_setopt(OFF_LFA_OPT_UNIQUE_ID) before joining.
 * Without a set id the provider falls back to a file rendezvous in
 * $OFF_LFA_BOOTSTRAP_DIR (rank 0 writes off_lfa-<key>.uid, the others poll
 * it; <key> = $OFF_LFA_BOOTSTRAP_KEY or "world").  A one-member set needs
 * neither.
 *
 * Transport.  By default the world group is an RCCL communicator over xGMI
 * and buffers may be device (or staged host) memory.  With
 * OFF_LFA_OPT_TRANSPORT = 1 (or OFF_LFA_TRANSPORT=peer) the provider instead
 * moves every transfer through the OWNER endpoint's tagged messaging with
 * FI_PEER_TRANSFER, as prov/coll does through rxm (coll_coll.c:770-814): the
 * owner must then provide fi_tsendmsg / fi_trecvmsg and report each finished
 * transfer through the peer_ops->complete this provider installs.  Host
 * buffers reduce in liblfa's host combine; device buffers (on the endpoint's
 * GPU, OFF_LFA_DEVICE) run the gfx950 kernels, with every transfer staged
 * through host memory so the owner only moves host bytes.  On a host without
 * a usable GPU (and no device named) the endpoint takes host buffers only.
 * No unique id is needed then.
 *
 * Environment: OFF_LFA_DEVICE (HIP device ordinal; default $LOCAL_RANK,
 * else 0; -1 with the peer transport: host buffers only, no GPU touched), OFF_LFA_PROGRESS=manual (no progress thread: the owner drives
 * progress through the util_ep progress slot or fi_cq_read on the
 * off_lfa CQ), OFF_LFA_ALGO (enum lfa_coll_algo), OFF_LFA_TRANSPORT=peer.
 */
#ifndef OFF_LFA_H
#define OFF_LFA_H

#define OFF_LFA_PROV_NAME "off_lfa"
#define FI_PROV_SPECIFIC_LFA (0x1fa << 16)

enum {
	/* 128 bytes (LFA_UNIQUE_ID_BYTES).  getopt: a fresh id (rank 0);
	 * setopt: the id every member bootstraps the world group with. */
	OFF_LFA_OPT_UNIQUE_ID = -FI_PROV_SPECIFIC_LFA,
	/* int: enum lfa_coll_algo (include/lfa_coll.h) */
	OFF_LFA_OPT_ALGO,
	/* size_t: host-buffer staging chunk in bytes (0 = default) */
	OFF_LFA_OPT_CHUNK,
	/* int: HIP device ordinal; only before the world join */
	OFF_LFA_OPT_DEVICE,
	/* int: 0 = RCCL over xGMI (default), 1 = the owner's peer transfers;
	 * only before the world join */
	OFF_LFA_OPT_TRANSPORT,
};

#endif /* OFF_LFA_H */
