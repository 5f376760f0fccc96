"""Lazy KV reservation (verdict r3 item 7): admission reserves the prompt + one block, decode runs grow the block
tables as contexts cross 64-token boundaries, an exhausted arena preempts the youngest running request (recompute on
re-admission).  CPU engine (fp32 reference ops) and the native scheduler; the Python fallback scheduler is held to
the same semantics."""
import pytest
import torch

from llm_based_apache_spark_optimization_amd.engine import SamplingParams, build_engine
from llm_based_apache_spark_optimization_amd.ops import reference as ref
from llm_based_apache_spark_optimization_amd.runtime import native


@pytest.mark.parametrize("impl", ["native", "python"])
def test_scheduler_grow_and_preempt(impl):
    cls = native.Scheduler if impl == "native" else native._PyScheduler
    s = cls(9, 64, 3, 10000, 8)  # 8 usable blocks, default reserve: one block of generation
    s.add(1, 100, 400)  # up front this would need 8 blocks; lazily 3 (100 + 64 tokens)
    s.add(2, 60, 400)
    s.add(3, 10, 10)
    assert s.admit() == [1, 2, 3]
    assert [len(s.block_table(i)) for i in (1, 2, 3)] == [3, 2, 1] and s.free_blocks == 2
    assert s.grow(1, 164) == 0            # already covered
    assert s.grow(1, 200) == 1 and len(s.block_table(1)) == 4
    assert s.grow(3, 10_000) == 0         # capped at prompt + max_new (20 tokens = 1 block)
    assert s.grow(2, 64 * 5) == -1        # needs 3 more, 1 free: nothing allocated
    assert s.free_blocks == 1 and len(s.block_table(2)) == 2
    assert s.youngest_first() == [3, 2, 1]
    s.preempt(3, 15, 5)                   # back to the FRONT of the queue with its resumed lengths
    assert s.num_running == 2 and s.num_waiting == 1 and s.free_blocks == 2
    s.add(4, 10, 10)
    assert s.grow(2, 64 * 4) == 2 and s.free_blocks == 0
    assert s.admit() == []                # no block for the resumed request 3
    s.finish(1)
    assert s.admit() == [3, 4]            # the preempted request is re-admitted first
    with pytest.raises(Exception):
        s.preempt(99, 1, 1)
    s.finish(2), s.finish(3), s.finish(4)
    assert s.free_blocks == 8 and s.num_running == 0


def test_option_less_requests_all_admitted():
    """32 option-less requests (Ollama's generate-until-EOS: max_tokens = the whole window) fit an arena of
    32 x (prompt + 256) tokens at once; reserving the window up front admits 8 of them."""
    prompt = list(range(1, 21))
    blocks = (32 * (len(prompt) + 256)) // 64 + 1
    for reserve, expect in ((64, 32), (-1, 8)):
        eng = build_engine("tiny-nsql", device="cpu", max_slots=32, max_model_len=1024, num_kv_blocks=blocks,
                           kv_reserve_tokens=reserve)
        reqs = [eng.add_request(prompt, SamplingParams.from_ollama_options({})) for _ in range(32)]
        assert all(q.params.max_tokens == 1024 - len(prompt) for q in reqs)
        eng.step()
        assert eng.sched.num_running == expect, (reserve, eng.sched.num_running)
        eng.abort_all("test over")
        assert eng.sched.free_blocks == blocks - 1


@pytest.fixture(scope="module")
def engines():
    kw = dict(device="cpu", max_slots=4, max_model_len=512, max_prefill_tokens=512)
    return (build_engine("tiny-nsql", kv_reserve_tokens=-1, **kw), build_engine("tiny-nsql", **kw))


def test_growth_decodes_like_reserve_up_front(engines):
    """A request whose output crosses several 64-token blocks decodes the same tokens with lazy growth as with the
    whole reservation up front (EOS-bounded runs of sync_every steps, so the tables grow many times)."""
    full, lazy = engines
    prompt = [1] + list(range(7, 37))
    sp = SamplingParams(max_tokens=220)  # EOS possible: runs of sync_every steps
    a = full.generate([prompt], sp)[0].token_ids
    b = lazy.generate([prompt], sp)[0].token_ids
    assert a == b
    assert lazy.stats["kv_grown_blocks"] >= (len(prompt) + len(b)) // 64 - 1
    assert lazy.sched.free_blocks == lazy.runner.num_kv_blocks - 1


def test_preemption_recomputes_identical_tokens():
    """An arena too small for every running request's growth: the youngest is preempted, re-admitted when a request
    retires, re-prefills its prompt + generated tokens, and every request still produces its solo greedy tokens."""
    prompts = [[1] + list(range(3 + k, 40 + k)) for k in range(3)]
    eng = build_engine("tiny-nsql", device="cpu", max_slots=3, max_model_len=512, num_kv_blocks=9)
    sp = SamplingParams(max_tokens=150, ignore_eos=True)
    solo = [eng.generate([p], sp)[0].token_ids for p in prompts]
    eng.run_ahead = 16  # decode runs of 16 steps: growth before each run
    reqs = [eng.add_request(p, sp) for p in prompts]
    eng.run_until_done(reqs)
    assert [q.output_ids for q in reqs] == solo
    assert eng.stats["preempted"] >= 1 and any(q.preemptions for q in reqs)
    assert all(len(q.output_ids) == 150 for q in reqs)
    assert eng.sched.free_blocks == 8 and eng.sched.num_running == 0


def test_preemption_keeps_seeded_sampling_stream():
    """Sampling at temperature > 0 with a fixed seed: a request that is preempted and re-admitted continues its
    random stream where it stopped (the resumed incarnation draws from counter offset len(resumed)).  Its tokens after the
    resume point follow the solo run's; they are compared over the first 8 only, because the re-prefill of the
    generated tokens rounds the bf16 activations differently from the incremental decode, and a later draw that
    lands near a CDF boundary may then flip (the unmodified stream diverges at once: every draw is shifted)."""
    prompts = [[1] + list(range(3 + k, 40 + k)) for k in range(3)]
    eng = build_engine("tiny-nsql", device="cpu", max_slots=3, max_model_len=512, num_kv_blocks=9)
    # the solo runs must decode on the batched runs' step: the batch-1 residual-reduce step rounds differently
    # (its row scale applies to the GEMM output, the norm-launch step's CPU path scales the bf16 input)
    eng.runner.rr_decode = False
    sps = [SamplingParams(max_tokens=150, ignore_eos=True, temperature=0.9, top_k=40, top_p=0.95, seed=100 + k)
           for k in range(3)]
    solo = [eng.generate([p], sp)[0].token_ids for p, sp in zip(prompts, sps)]
    eng.run_ahead = 16
    reqs = [eng.add_request(p, sp) for p, sp in zip(prompts, sps)]
    eng.run_until_done(reqs)
    assert eng.stats["preempted"] >= 1 and any(q.preemptions for q in reqs)
    for q, s in zip(reqs, solo):
        if not q.preemptions:
            assert q.output_ids == s
        else:
            n = len(q.resumed) + 8
            assert q.output_ids[:n] == s[:n]


def test_sampler_stream_keyed_by_seed_with_counter_offset():
    """The reference sampler's draw for step g of a row comes from (seed key, g + offset) alone: a resumed request
    (offset R) continues its stream, (key, R, g) == (key, 0, g + R), whatever the other rows of the batch are; and
    neighbouring keys are NOT shifted copies of one stream (seed s + 1 at step g used to equal seed s at g + 1)."""
    torch.manual_seed(0)
    V, B = 300, 3
    logits = torch.randn(B, V)
    args = dict(temperature=torch.full((B,), 0.9), top_k=torch.full((B,), 50, dtype=torch.int32),
                top_p=torch.full((B,), 0.95))

    def draw(seeds, gl):
        st = [torch.zeros(B, 32, dtype=torch.int32), torch.tensor(gl, dtype=torch.int32),
              torch.zeros(B, dtype=torch.int32), torch.zeros(B, dtype=torch.int32), torch.zeros(B, dtype=torch.int32)]
        ref.sample_commit(logits.clone(), None, None, args["temperature"], args["top_k"], args["top_p"],
                          torch.tensor(seeds), st[0], st[1], st[2], st[3], st[4], torch.tensor([-1]))
        return [int(st[0][b, gl[b]]) for b in range(B)]

    toks = [draw([ref.pack_seed(7, R), 11, 13], [3, 0, 0])[0] for R in range(20)]
    assert toks == [draw([7, 11, 13], [3 + R, 0, 0])[0] for R in range(20)]
    assert draw([7, 11, 13], [3, 0, 0])[0] == draw([7, 99, 5], [3, 2, 1])[0]
    assert all(ref.draw_seed(s + 1, g) != ref.draw_seed(s, g + 1) for s in range(50) for g in range(20))
    shifted = [draw([8, 11, 13], [g, 0, 0])[0] == draw([7, 11, 13], [g + 1, 0, 0])[0] for g in range(20)]
    assert sum(shifted) < 15


def test_admission_hold_clears_on_free_blocks():
    """After a preemption the engine holds admissions only until enough KV blocks are free for the preempted
    request plus one block of growth per running request, not until a running request retires."""
    eng = build_engine("tiny-nsql", device="cpu", max_slots=3, max_model_len=512, num_kv_blocks=9)
    eng._admit_hold, eng._admit_hold_blocks = True, 1
    q = eng.add_request([1, 5, 6, 7], SamplingParams(max_tokens=4, ignore_eos=True))
    eng.run_until_done([q])
    assert not eng._admit_hold and len(q.output_ids) == 4
