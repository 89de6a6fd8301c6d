"""Oracle (test infrastructure only): the run merge of egs/alimeeting/umap_cluster/make_rttm.py
(merge_segments, :49-73) as the reference's sequential loop, restated, to check the product's
vectorised merge (speaker_diarization_amd/cluster/spectral.py) on random sub-segment streams beyond
the reference-run goldens."""


def merge_segments_seq(utt_to_subs):
    out = []
    for utt, subs in utt_to_subs.items():
        if not subs:
            continue
        cur_b, cur_e, cur_l = subs[0]
        last_e = cur_e
        for b, e, la in subs[1:]:
            last_e = e
            if b <= cur_e and la == cur_l:          # touching / overlapping, same label: extend
                cur_e = e
            elif b > cur_e:                         # gap: close at the open segment's end
                out.append((utt, cur_b, cur_e, cur_l))
                cur_b, cur_e, cur_l = b, e, la
            else:                                   # overlap, new label: split at the midpoint
                mid = (b + cur_e) / 2.0
                out.append((utt, cur_b, mid, cur_l))
                cur_b, cur_e, cur_l = mid, e, la
        out.append((utt, cur_b, last_e, cur_l))
    return out
