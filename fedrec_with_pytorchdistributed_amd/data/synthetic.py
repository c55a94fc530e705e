"""Synthetic MIND-format shards with a planted, learnable signal.

The reference ships a one-user toy shard and no MIND preprocessing (C33), and there is no
network here, so every benchmark and quality run uses data from this generator.  It emits
the exact reference file formats (§2.6), so the reference code could consume the same
files for an A/B comparison.

Signal model (learnable through a *random-init frozen* backbone):

* ``K`` topics, each owning a disjoint set of "topic word" ids; a title draws most of its
  words from its topic's set, the rest from a shared pool of common words.
* Each news item has a topic and a Zipf popularity inside its topic.
* Each user has a peaky Dirichlet preference over topics; history items and positives are
  drawn from it, negatives mostly from the complementary topic mass.

Titles are ``[101, w_1..w_L, 102, 0 ...]`` padded to ``T=50`` with mask ``1`` over the
first ``L+2`` positions (``L`` in ``[3, 36]``: the shipped shard's mask lengths are
0-38, mean 16.3 -- E1).  Row 0 is the all-zero ``<unk>``/pad row.

Everything is vectorised numpy and deterministic in ``(seed, client)``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .shard import ImpressionArrays, Shard

CLS, SEP = 101, 102


@dataclass
class SynthSpec:
    num_news: int = 65_000  # MIND-small has ~65k news
    num_users: int = 50_000  # ~50k users
    num_topics: int = 20
    title_len: int = 50
    # 48 topic words per topic (960 in all): with the backbone frozen at random init each word
    # is a random 768-d vector, so the head can only map words to topics linearly when the
    # topic vocabulary is not much larger than the width.  A linear probe on the mean token
    # vector recovers the topic of held-out titles 98 % of the time at 40 words/topic but
    # 58 % at 400 (the first default, whose quality runs stayed at AUC ~0.5).
    words_per_topic: int = 48
    common_words: int = 4000
    topic_word_prob: float = 0.6
    title_len_mean: float = 14.0
    title_len_std: float = 5.0
    his_len_mean: float = 30.0  # lognormal-ish; some histories exceed 50 (exercise Q6)
    his_len_max: int = 90
    imps_per_user: float = 3.0
    negs_mean: float = 24.0
    negs_max: int = 150
    dirichlet_alpha: float = 0.25
    neg_other_topic: float = 0.85
    zipf_s: float = 1.0
    valid_frac: float = 0.2
    seed: int = 0

    @staticmethod
    def preset(name: str) -> "SynthSpec":
        if name == "toy":  # shipped-shard scale (E1): 1 user, 4+1 impressions, ~224 news
            return SynthSpec(num_news=224, num_users=1, imps_per_user=4.0, negs_mean=143,
                             negs_max=143, his_len_mean=76, his_len_max=76, valid_frac=1.0)
        if name == "tiny":
            return SynthSpec(num_news=2000, num_users=300, num_topics=8)
        if name == "small":  # quick CPU runs
            return SynthSpec(num_news=8000, num_users=4000, num_topics=12)
        if name in ("mind-small", "mind_small"):
            return SynthSpec()
        if name in ("mind-large", "mind_large"):
            return SynthSpec(num_news=161_000, num_users=1_000_000)
        raise ValueError(f"unknown synthetic preset {name!r}")


class SyntheticCorpus:
    """The global news corpus + users; clients are disjoint user subsets."""

    def __init__(self, spec: SynthSpec):
        self.spec = spec
        rng = np.random.Generator(np.random.PCG64(spec.seed))
        K, N = spec.num_topics, spec.num_news
        # disjoint vocabularies: topic words from [1000, 29000), common words after them
        pool = rng.permutation(np.arange(1000, 29600))
        tw = spec.words_per_topic
        self.topic_words = pool[: K * tw].reshape(K, tw)
        self.common = pool[K * tw: K * tw + spec.common_words]
        # news topics and titles (row 0 = <unk>)
        self.news_topic = np.concatenate([[-1], rng.integers(0, K, N)])
        L = np.clip(np.rint(rng.normal(spec.title_len_mean, spec.title_len_std, N)), 3, 36).astype(np.int64)
        T = spec.title_len
        tok = np.zeros((N + 1, 2, T), dtype=np.int64)
        pos = np.arange(T)[None, :]
        is_topic = rng.random((N, T)) < spec.topic_word_prob
        tw_pick = self.topic_words[self.news_topic[1:, None], rng.integers(0, tw, (N, T))]
        cw_pick = self.common[rng.integers(0, len(self.common), (N, T))]
        words = np.where(is_topic, tw_pick, cw_pick)
        body = np.where(pos < L[:, None] + 1, np.roll(words, 1, axis=1), 0)
        body[:, 0] = CLS
        body = np.where(pos == L[:, None] + 1, SEP, body)
        tok[1:, 0, :] = body
        tok[1:, 1, :] = (pos < L[:, None] + 2).astype(np.int64)
        self.news_index = tok
        # popularity: Zipf within topic; cumulative table for a single vectorised sampler
        self._by_topic = [np.nonzero(self.news_topic == k)[0] for k in range(K)]
        cums, offs = [], []
        for k in range(K):
            n = len(self._by_topic[k])
            w = 1.0 / np.power(rng.permutation(n) + 1.0, spec.zipf_s)
            c = np.cumsum(w)
            cums.append(k + c / c[-1])
            offs.append(n)
        self._cum = np.concatenate(cums)
        self._flat = np.concatenate(self._by_topic)
        self._topic_start = np.concatenate([[0], np.cumsum(offs)])

    # ------------------------------------------------------------------------------
    def _draw_news(self, rng: np.random.Generator, topics: np.ndarray) -> np.ndarray:
        u = topics + rng.random(topics.shape) * 0.999999
        j = np.searchsorted(self._cum, u, side="left")
        return self._flat[np.minimum(j, len(self._flat) - 1)]

    @staticmethod
    def _draw_topics(rng: np.random.Generator, probs: np.ndarray, counts: np.ndarray) -> np.ndarray:
        """Draw ``counts[i]`` topics from row ``probs[i]`` (flattened output)."""
        rows = np.repeat(np.arange(len(counts)), counts)
        c = np.cumsum(probs, axis=1)
        u = rng.random(len(rows)) * c[rows, -1]
        return (u[:, None] > c[rows]).sum(axis=1)

    def users(self, client: int, num_clients: int) -> np.ndarray:
        return np.arange(client, self.spec.num_users, num_clients)

    def client_shard(self, client: int = 0, num_clients: int = 1,
                     full_news_table: bool = False) -> Shard:
        spec = self.spec
        rng = np.random.Generator(np.random.PCG64([spec.seed, 7919 + client]))
        users = self.users(client, num_clients)
        U, K = len(users), spec.num_topics
        pref = rng.dirichlet(np.full(K, spec.dirichlet_alpha), U)
        # history per user
        hl = np.clip(np.rint(rng.lognormal(np.log(spec.his_len_mean), 0.6, U)), 1,
                     spec.his_len_max).astype(np.int64)
        his_topics = self._draw_topics(rng, pref, hl)
        his_all = self._draw_news(rng, his_topics)
        his_ptr_u = np.concatenate([[0], np.cumsum(hl)])
        # impressions per user: train + (maybe) one valid
        n_imp = 1 + rng.poisson(max(spec.imps_per_user - 1, 0), U)
        has_valid = rng.random(U) < spec.valid_frac
        tot = n_imp + has_valid
        imp_user = np.repeat(np.arange(U), tot)
        I = len(imp_user)
        pos = self._draw_news(rng, self._draw_topics(rng, pref[imp_user], np.ones(I, np.int64)))
        nn = np.clip(rng.poisson(spec.negs_mean, I), 4, spec.negs_max).astype(np.int64)
        other = (1.0 - pref) / np.maximum((1.0 - pref).sum(1, keepdims=True), 1e-9)
        negp = spec.neg_other_topic * other + (1 - spec.neg_other_topic) / K
        neg_topics = self._draw_topics(rng, negp[imp_user], nn)
        negs = self._draw_news(rng, neg_topics)
        neg_ptr = np.concatenate([[0], np.cumsum(nn)])
        # the last impression of a user with has_valid goes to the validation split
        last_of_user = np.concatenate([np.diff(imp_user) != 0, [True]])
        is_valid = last_of_user & has_valid[imp_user]

        def build(mask: np.ndarray):
            idx = np.nonzero(mask)[0]
            his_len = hl[imp_user[idx]]
            hp = np.concatenate([[0], np.cumsum(his_len)])
            his_ids = np.concatenate([his_all[his_ptr_u[u]:his_ptr_u[u + 1]] for u in imp_user[idx]]) \
                if len(idx) else np.zeros(0, np.int64)
            nlen = nn[idx]
            npt = np.concatenate([[0], np.cumsum(nlen)])
            neg_ids = np.concatenate([negs[neg_ptr[i]:neg_ptr[i + 1]] for i in idx]) \
                if len(idx) else np.zeros(0, np.int64)
            return pos[idx], npt, neg_ids, hp, his_ids, imp_user[idx]

        tr = build(~is_valid)
        va = build(is_valid)
        # local news table: only the news this client references (+ row 0), like UserData
        if full_news_table:
            local = np.arange(len(self.news_index))
        else:
            local = np.unique(np.concatenate([[0], tr[0], tr[2], tr[4], va[0], va[2], va[4]]))
        remap = np.zeros(len(self.news_index), dtype=np.int64)
        remap[local] = np.arange(len(local))
        news_index = self.news_index[local]
        index2nid = ["<unk>"] + [f"N{int(g)}" for g in local[1:]]
        nid2index = {n: i for i, n in enumerate(index2nid)}

        def arrays(t) -> ImpressionArrays:
            p, npt, nids, hp, hids, u = t
            return ImpressionArrays(remap[p].astype(np.int32), npt.astype(np.int64),
                                    remap[nids].astype(np.int32), hp.astype(np.int64),
                                    remap[hids].astype(np.int32), u.astype(np.int32))

        uids = [f"U{int(users[u])}" for u in range(U)]
        return Shard(news_index, nid2index, arrays(tr), arrays(va), None, index2nid, uids)


def make_client_shards(preset: str = "small", num_clients: int = 1, seed: int = 0,
                       full_news_table: bool = False, spec: Optional[SynthSpec] = None) -> List[Shard]:
    spec = spec or SynthSpec.preset(preset)
    spec.seed = seed
    corpus = SyntheticCorpus(spec)
    return [corpus.client_shard(k, num_clients, full_news_table) for k in range(num_clients)]


def write_client_dirs(root: str, preset: str = "small", num_clients: int = 1, seed: int = 0) -> List[str]:
    """Write ``root/client{k}/`` reference-layout directories; return their paths."""
    import os

    out = []
    for k, s in enumerate(make_client_shards(preset, num_clients, seed)):
        d = os.path.join(root, f"client{k}")
        s.save(d)
        out.append(d)
    return out
