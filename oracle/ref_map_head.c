/*
 * TEST INFRASTRUCTURE ONLY -- never linked into libbcp.
 *
 * `make ref` builds oracle/_ref/ref_map_targets, a small program, from ONE
 * translation unit: the reference's text streamed unchanged from
 * /root/reference (ref_stream.sh, SHA-checked, no copy written) --
 *
 *   common/common.h:15-34, 44-48    FileInfo & bit macros, Target, RunData
 *   gen/main.c:50-52                st2rank, rank2st, st_weight
 *
 * then this head, then the coordinator's own mapping code of gen/main.c
 * (rank 0 after the MPI_Gathers):
 *
 *   gen/main.c:498-499              "Fewer targets than last run"
 *   gen/main.c:506-541              previous list kept, new targets appended,
 *                                   st2rank / rank2st / st_weight
 *
 * streamed into the body of run_map() below, then ref_map_tail.c.  errx is
 * the C library's own: on the reference's fatal checks the program prints
 * the reference's message and exits 1, as bp-parity-gen would.  The glue
 * sets up only what MPI_Gather would have delivered (gen/main.c:487-496:
 * world rank 2r+1 the eater and 2r+2 the feeder of host r, both with that
 * host's targetNumID; lines 500-505 check exactly that layout) and the
 * previous run's list (RunData read from spool/data, :464-470).
 *
 *   ref_map_targets <nprev> <prev ids...> <ntargets> <ids in rank order...>
 *   -> "st_ids ...", "st2rank ...", "round_st ..." (round r = communicator
 *      rank r+1 = world rank 2r+1, :570-574, :758: rank2st[2r+1])
 */
#include <stdio.h>

static void run_map(int nprev, const int *prev_ids, int ntargets, const int *rank_ids)
{
    RunData last_run;
    memset(&last_run, 0, sizeof(last_run));
    last_run.ntargets = nprev;
    for (int i = 0; i < nprev; i++) {
        last_run.targetIDs[i].id = prev_ids[i];
        last_run.targetIDs[i].rank = -1;
    }
    Target targetIDs[2 * MAX_STORAGE_TARGETS + 1];
    int target_weights[2 * MAX_STORAGE_TARGETS + 1];
    memset(targetIDs, 0, sizeof(targetIDs));
    memset(target_weights, 0, sizeof(target_weights));
    for (int r = 0; r < ntargets; r++) {
        targetIDs[2 * r + 1] = (Target){rank_ids[r], 2 * r + 1, 0};
        targetIDs[2 * r + 2] = (Target){rank_ids[r], 2 * r + 2, 0};
        target_weights[2 * r + 1] = 1000 + r;
    }
