"""Topic models: ``train_lda`` / ``lda_predict`` (online variational Bayes LDA, Hoffman et al.
NIPS'10) and ``train_plsa`` / ``plsa_predict`` (incremental EM pLSA).

Reference behaviour: Hivemall LDAUDTF, OnlineLDAModel, LDAPredictUDAF, PLSAUDTF,
IncrementalPLSAModel, PLSAPredictUDAF (upstream core/src/main/java/hivemall/topicmodel/;
SURVEY.md §2.3.7, K11).

Device design: a mini-batch of documents is flattened to (doc, word, count) non-zeros and the
E-step runs vectorised over all of them (gather of exp E[log β] columns, scatter-add per
document) — on the GPU it is a handful of fused torch kernels per inner iteration.  The
vocabulary is dictionary-encoded on the host (words are strings in SQL).

Model tables: LDA ``(label int, word string, lambda float)``; pLSA ``(label, word, prob)``.
"""
from __future__ import annotations

import math
import os

import numpy as np
import pandas as pd
import torch

from .. import _native
from ..registry import udaf
from ..utils.options import UDFArgumentException, opt
from .base import Learner, log

_native.register_hip("hm_lda_estep", [_native.c_p, _native.c_p, _native.c_p, _native.c_p, _native.c_int,
                                      _native.c_int, _native.c_f32, _native.c_f32, _native.c_int,
                                      _native.c_p, _native.c_p, _native.c_p, _native.c_p])

LDA_OPTS = [
    opt("topics", "k", 10, int, "Number of topics"),
    opt("alpha", None, None, float, "Document-topic prior (default 1/topics)"),
    opt("eta", None, None, float, "Topic-word prior (default 1/topics)"),
    opt("num_docs", "d", -1, int, "Total number of documents (default: #docs)"),
    opt("tau0", None, 64.0, float, "Learning-rate delay"),
    opt("kappa", None, 0.7, float, "Learning-rate exponent"),
    opt("iters", "iterations", 10, int, "Epochs", aliases=("iter",)),
    opt("delta", None, 1e-3, float, "E-step convergence threshold (mean |Δγ|)"),
    opt("eps", None, 1e-1, float, "Perplexity convergence threshold"),
    opt("mini_batch_size", "batch_size", 128, int, "Documents per mini-batch"),
    opt("max_inner_iters", None, 100, int, "[engine] E-step iteration cap"),
    opt("seed", None, -1, int, "Seed"),
]


def _parse_doc(doc) -> dict:
    """['word', 'word:count', ...] or a {word: count} map -> {word: count}."""
    out: dict = {}
    if doc is None:
        return out
    if isinstance(doc, dict):
        return {str(k): float(v) for k, v in doc.items()}
    for t in doc:
        s = str(t)
        p = s.rfind(":")
        if p > 0:
            try:
                out[s[:p]] = out.get(s[:p], 0.0) + float(s[p + 1:])
                continue
            except ValueError:
                pass
        out[s] = out.get(s, 0.0) + 1.0
    return out


class _Vocab:
    def __init__(self):
        self.ids: dict = {}
        self.words: list = []

    def encode(self, docs, add=True):
        rows = []
        for d in docs:
            r = []
            for w, c in _parse_doc(d).items():
                i = self.ids.get(w)
                if i is None and add:
                    i = self.ids[w] = len(self.words)
                    self.words.append(w)
                if i is not None:
                    r.append((i, c))
            rows.append(r)
        return rows


def _flatten(rows, device):
    """[(word id, count)] rows -> (doc, word, count) tensors, built with numpy (no per-token
    torch calls)."""
    lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=len(rows))
    n = int(lens.sum())
    doc = np.repeat(np.arange(len(rows), dtype=np.int64), lens)
    w = np.fromiter((i for r in rows for i, _ in r), dtype=np.int64, count=n)
    c = np.fromiter((x for r in rows for _, x in r), dtype=np.float32, count=n)
    t = lambda a: torch.from_numpy(a).to(device)
    return t(doc), t(w), t(c)


class LDA(Learner):
    NAME = "train_lda"
    OPTIONS = LDA_OPTS

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        c = self.cl
        self.K = int(c["topics"])
        if self.K < 1:
            raise UDFArgumentException("train_lda: -topics must be >= 1")
        self.alpha = c["alpha"] if c["alpha"] is not None else 1.0 / self.K
        self.eta = c["eta"] if c["eta"] is not None else 1.0 / self.K
        self.vocab = _Vocab()
        self.lam: torch.Tensor | None = None
        self.t = 0
        self.gen = torch.Generator(device="cpu").manual_seed(self.seed)

    def _grow(self, V):
        dev = self.device
        if self.lam is None:
            self.lam = torch.distributions.Gamma(100.0, 100.0).sample((self.K, V)).to(dev)
        elif self.lam.shape[1] < V:
            extra = torch.distributions.Gamma(100.0, 100.0).sample((self.K, V - self.lam.shape[1])).to(dev)
            self.lam = torch.cat([self.lam, extra], 1)

    def _elog(self, x: torch.Tensor, dim: int) -> torch.Tensor:
        return torch.digamma(x) - torch.digamma(x.sum(dim, keepdim=True))

    def e_step(self, doc, w, c, B, expElogbeta):
        """Per-document fixed point of gamma (upstream OnlineLDAModel.eStep: each document
        iterates until mean |Δγ| < -delta).  GPU: one fused gfx950 kernel for the whole loop
        (csrc/kernels/lda.hip); CPU: the same iteration as torch ops with a per-document
        convergence mask."""
        c_ = self.cl
        gamma = torch.distributions.Gamma(100.0, 100.0).sample((B, self.K)).to(self.device)
        if self.device.type == "cuda" and self.K <= 256 and os.environ.get("HM_LDA_TORCH", "0") != "1":
            return self._e_step_kernel(doc, w, c, B, expElogbeta, gamma)
        Eb = expElogbeta[:, w].T                                  # [N, K]
        active = torch.ones(B, dtype=torch.bool, device=self.device)
        for _ in range(int(c_["max_inner_iters"])):
            Et = torch.exp(self._elog(gamma, 1))                  # [B, K]
            phinorm = (Et[doc] * Eb).sum(1) + 1e-30               # [N]
            contrib = Et[doc] * Eb * (c / phinorm)[:, None]       # [N, K]
            new = torch.full((B, self.K), float(self.alpha), device=self.device)
            new.index_add_(0, doc, contrib)
            change = (new - gamma).abs().mean(1)
            gamma = torch.where(active[:, None], new, gamma)
            active &= change >= c_["delta"]
            if not bool(active.any()):
                break
        Et = torch.exp(self._elog(gamma, 1))
        phinorm = (Et[doc] * Eb).sum(1) + 1e-30
        contrib = Et[doc] * Eb * (c / phinorm)[:, None]
        return gamma, contrib

    def _e_step_kernel(self, doc, w, c, B, expElogbeta, gamma):
        from .. import _native

        dev = self.device
        off = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        off[1:] = torch.cumsum(torch.bincount(doc, minlength=B), 0).to(torch.int32)
        EbT = expElogbeta.T.contiguous()                          # [V, K]: a word's row contiguous
        wid = w.to(torch.int32).contiguous()
        cc = c.to(torch.float32).contiguous()
        gamma = gamma.contiguous()
        contrib = torch.empty((w.numel(), self.K), dtype=torch.float32, device=dev)
        self.inner_iters = torch.zeros(B, dtype=torch.int32, device=dev)
        p = _native.ptr
        rc = _native.hip().hm_lda_estep(p(off), p(wid), p(cc), p(EbT), B, self.K, float(self.alpha),
                                        float(self.cl["delta"]), int(self.cl["max_inner_iters"]), p(gamma),
                                        p(contrib), p(self.inner_iters), _native.stream_of(dev))
        _native.check(rc, "hm_lda_estep")
        return gamma, contrib

    def fit(self, docs) -> "LDA":
        c = self.cl
        rows = self.vocab.encode(list(docs), add=True)
        V = len(self.vocab.words)
        self._grow(V)
        D = c["num_docs"] if c["num_docs"] > 0 else len(rows)
        bs = int(c["mini_batch_size"])
        prev = None
        # the corpus flattened ONCE to device CSR (doc, word, count); mini-batches are slices
        doc_all, w_all, c_all = _flatten(rows, self.device)
        ptr = np.zeros(len(rows) + 1, dtype=np.int64)
        np.cumsum([len(r) for r in rows], out=ptr[1:])
        total = float(c_all.sum().item()) if c_all.numel() else 0.0
        for ep in range(int(c["iters"])):
            bound = torch.zeros((), dtype=torch.float64, device=self.device)
            for s in range(0, len(rows), bs):
                e = min(len(rows), s + bs)
                a, b = int(ptr[s]), int(ptr[e])
                batch = rows[s:e]
                doc, w, cnt = doc_all[a:b] - s, w_all[a:b], c_all[a:b]
                if doc.numel() == 0:
                    continue
                expElogbeta = torch.exp(self._elog(self.lam, 1))
                gamma, contrib = self.e_step(doc, w, cnt, len(batch), expElogbeta)
                sstats = torch.zeros_like(self.lam)
                sstats.index_add_(1, w, contrib.T)
                rho = (c["tau0"] + self.t) ** (-c["kappa"])
                self.lam = (1 - rho) * self.lam + rho * (self.eta + D / len(batch) * sstats)
                self.t += 1
                bound -= (cnt * torch.log((torch.exp(self._elog(gamma, 1))[doc] *
                                           expElogbeta[:, w].T).sum(1) + 1e-100)).sum().double()
            ppl = math.exp(float(bound.item()) / max(1.0, total))       # one sync per epoch
            log.info("train_lda epoch %d perplexity %.3f", ep + 1, ppl)
            if prev is not None and abs(prev - ppl) < c["eps"]:
                break
            prev = ppl
        self.perplexity = prev
        return self

    def topic_word(self, normalize: bool = True) -> torch.Tensor:
        return self.lam / self.lam.sum(1, keepdim=True) if normalize else self.lam

    def model_table(self) -> pd.DataFrame:
        L = self.lam.cpu().numpy()
        K, V = L.shape
        return pd.DataFrame({"label": np.repeat(np.arange(K), V), "word": self.vocab.words * K,
                             "lambda": L.reshape(-1)})

    def transform(self, docs) -> np.ndarray:
        rows = self.vocab.encode(list(docs), add=False)
        doc, w, cnt = _flatten(rows, self.device)
        expElogbeta = torch.exp(self._elog(self.lam, 1))
        gamma, _ = self.e_step(doc, w, cnt, len(rows), expElogbeta)
        return (gamma / gamma.sum(1, keepdim=True)).cpu().numpy()


@udaf("lda_predict")
def lda_predict(words, values, labels, lambdas, options=None):
    """Topic distribution of one document from the joined (word, count, topic, lambda) rows:
    returns [(label, probability)] sorted by probability."""
    o = options[0] if isinstance(options, (list, tuple)) and options else options
    K = None
    if o:
        toks = str(o).split()
        if "-topics" in toks:
            K = int(toks[toks.index("-topics") + 1])
    K = K or (max(int(l) for l in labels if l is not None) + 1)
    lam: dict = {}
    cnt: dict = {}
    for wd, v, l, la in zip(words, values, labels, lambdas):
        if wd is None or l is None:
            continue
        lam.setdefault(wd, np.zeros(K))[int(l)] = float(la)
        cnt[wd] = float(v) if v is not None else 1.0
    if not lam:
        return []
    m = LDA(f"-topics {K}", device="cpu")
    words_ = list(lam)
    m.vocab.words = words_
    m.vocab.ids = {w: i for i, w in enumerate(words_)}
    m.lam = torch.tensor(np.stack([lam[w] for w in words_], 1), dtype=torch.float32).clamp_min(1e-10)
    theta = m.transform([{w: cnt[w] for w in words_}])[0]
    return sorted(((int(k), float(p)) for k, p in enumerate(theta)), key=lambda kv: -kv[1])


PLSA_OPTS = [
    opt("topics", "k", 10, int, "Number of topics"),
    opt("alpha", None, 0.5, float, "Learning rate of the incremental P(w|z) update"),
    opt("delta", None, 1e-3, float, "Convergence threshold of the per-document EM"),
    opt("iters", "iterations", 10, int, "Epochs", aliases=("iter",)),
    opt("eps", None, 1e-1, float, "Perplexity convergence threshold"),
    opt("mini_batch_size", "batch_size", 128, int, "Documents per mini-batch"),
    opt("seed", None, -1, int, "Seed"),
]


class PLSA(Learner):
    NAME = "train_plsa"
    OPTIONS = PLSA_OPTS

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        self.K = int(self.cl["topics"])
        self.vocab = _Vocab()
        self.pwz: torch.Tensor | None = None       # [K, V]
        self.gen = torch.Generator(device="cpu").manual_seed(self.seed)

    def _grow(self, V):
        if self.pwz is None:
            p = torch.rand(self.K, V, generator=self.gen) + 0.5
            self.pwz = (p / p.sum(1, keepdim=True)).to(self.device)
        elif self.pwz.shape[1] < V:
            extra = torch.full((self.K, V - self.pwz.shape[1]), 1e-6, device=self.device)
            self.pwz = torch.cat([self.pwz, extra], 1)
            self.pwz /= self.pwz.sum(1, keepdim=True)

    def _doc_em(self, doc, w, c, B, iters=50):
        pzd = torch.full((B, self.K), 1.0 / self.K, device=self.device)
        Pw = self.pwz[:, w].T                                      # [N, K]
        for _ in range(iters):
            q = pzd[doc] * Pw
            q = q / q.sum(1, keepdim=True).clamp_min(1e-30)        # p(z | d, w)
            new = torch.zeros_like(pzd).index_add_(0, doc, q * c[:, None])
            new = new / new.sum(1, keepdim=True).clamp_min(1e-30)
            ch = float((new - pzd).abs().mean().item())
            pzd = new
            if ch < self.cl["delta"]:
                break
        q = pzd[doc] * Pw
        q = q / q.sum(1, keepdim=True).clamp_min(1e-30)
        return pzd, q

    def fit(self, docs) -> "PLSA":
        c = self.cl
        rows = self.vocab.encode(list(docs), add=True)
        self._grow(len(self.vocab.words))
        bs = int(c["mini_batch_size"])
        a = float(c["alpha"])
        for ep in range(int(c["iters"])):
            for s in range(0, len(rows), bs):
                doc, w, cnt = _flatten(rows[s:s + bs], self.device)
                if doc.numel() == 0:
                    continue
                _, q = self._doc_em(doc, w, cnt, len(rows[s:s + bs]))
                nwz = torch.zeros_like(self.pwz).index_add_(1, w, (q * cnt[:, None]).T)
                upd = nwz / nwz.sum(1, keepdim=True).clamp_min(1e-30)
                self.pwz = (1 - a) * self.pwz + a * upd
                self.pwz = self.pwz / self.pwz.sum(1, keepdim=True)
        return self

    def model_table(self) -> pd.DataFrame:
        P = self.pwz.cpu().numpy()
        K, V = P.shape
        return pd.DataFrame({"label": np.repeat(np.arange(K), V), "word": self.vocab.words * K,
                             "prob": P.reshape(-1)})

    def transform(self, docs) -> np.ndarray:
        rows = self.vocab.encode(list(docs), add=False)
        doc, w, cnt = _flatten(rows, self.device)
        pzd, _ = self._doc_em(doc, w, cnt, len(rows))
        return pzd.cpu().numpy()


@udaf("plsa_predict")
def plsa_predict(words, values, labels, probs, options=None):
    o = options[0] if isinstance(options, (list, tuple)) and options else options
    K = None
    if o:
        toks = str(o).split()
        if "-topics" in toks:
            K = int(toks[toks.index("-topics") + 1])
    K = K or (max(int(l) for l in labels if l is not None) + 1)
    pw: dict = {}
    cnt: dict = {}
    for wd, v, l, p in zip(words, values, labels, probs):
        if wd is None or l is None:
            continue
        pw.setdefault(wd, np.full(K, 1e-10))[int(l)] = float(p)
        cnt[wd] = float(v) if v is not None else 1.0
    if not pw:
        return []
    m = PLSA(f"-topics {K}", device="cpu")
    ws = list(pw)
    m.vocab.words, m.vocab.ids = ws, {w: i for i, w in enumerate(ws)}
    m.pwz = torch.tensor(np.stack([pw[w] for w in ws], 1), dtype=torch.float32)
    theta = m.transform([{w: cnt[w] for w in ws}])[0]
    return sorted(((int(k), float(p)) for k, p in enumerate(theta)), key=lambda kv: -kv[1])


def register_sql(reg):
    def one_arg(cls):
        class W(cls):
            def fit(self, docs, *_):
                return cls.fit(self, docs)
        W.__name__ = cls.__name__
        return W
    reg("train_lda", lambda: one_arg(LDA), n_data_args=1)
    reg("train_plsa", lambda: one_arg(PLSA), n_data_args=1)
