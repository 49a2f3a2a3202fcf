"""The CLIP BPE tokenizer (clap2diffusion_amd/tokenizer.py) against transformers'
CLIPTokenizer -- the tokenizer of the SD1.5 pipeline the reference drives -- on a synthetic
vocab.json / merges.txt pair learned here from a small corpus (the real SD1.5 files are not
available offline).  transformers is imported by this test only, never by the product."""
import collections
import json

import pytest
import torch

from clap2diffusion_amd.tokenizer import CLIPBPETokenizer, bytes_to_unicode

CORPUS = """a beach at sunset with waves crashing on the shore, thunder and rain over the city
a dog barking in the forest while birds are singing; people talking in a busy street
the sound of an engine, a helicopter flying overhead and sirens in the distance
it's raining heavily -- we're near 3 rivers and 42 bridges! they'll see the storm's eye""".split()


def learn_bpe(words, n_merges):
    b2u = bytes_to_unicode()
    freq = collections.Counter("".join(b2u[b] for b in w.lower().encode()) for w in words)
    seqs = {w: list(w[:-1]) + [w[-1] + "</w>"] for w in freq}
    merges = []
    for _ in range(n_merges):
        pairs = collections.Counter()
        for w, s in seqs.items():
            for a, b in zip(s, s[1:]):
                pairs[(a, b)] += freq[w]
        if not pairs:
            break
        (a, b), _ = max(pairs.items(), key=lambda kv: (kv[1], kv[0]))
        merges.append((a, b))
        for w, s in seqs.items():
            out, i = [], 0
            while i < len(s):
                if i < len(s) - 1 and s[i] == a and s[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(s[i])
                    i += 1
            seqs[w] = out
    chars = list(b2u.values())
    vocab = chars + [c + "</w>" for c in chars] + ["".join(m) for m in merges] + ["<|startoftext|>", "<|endoftext|>"]
    return {t: i for i, t in enumerate(dict.fromkeys(vocab))}, merges


@pytest.fixture(scope="module")
def tok_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("clip_tok")
    vocab, merges = learn_bpe(CORPUS, 220)
    (d / "vocab.json").write_text(json.dumps(vocab), encoding="utf-8")
    (d / "merges.txt").write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n",
                                  encoding="utf-8")
    (d / "special_tokens_map.json").write_text(json.dumps({"pad_token": "<|endoftext|>"}), encoding="utf-8")
    return d


PROMPTS = ["a beach", "", "A Beach At SUNSET", "thunder  and\train\nover the city", "it's raining; we're near 3 rivers!",
           "the storm's eye -- 42 bridges, 7 dogs.", "café naïve résumé 東京 thunder", "unseenwordxyz qqq zzz",
           " ".join(["waves"] * 90), "<|startoftext|>a dog<|endoftext|>", "sirens...!!! (distance) [helicopter]"]


@pytest.mark.parametrize("prompt", PROMPTS)
def test_bpe_matches_transformers_clip_tokenizer(tok_dir, prompt):
    from transformers.models.clip.tokenization_clip import CLIPTokenizer
    ref = CLIPTokenizer.from_pretrained(str(tok_dir))
    ours = CLIPBPETokenizer.from_folder(tok_dir)
    want = ref(prompt, padding="max_length", max_length=77, truncation=True).input_ids
    got = ours.ids(prompt)
    assert got == want
    assert ours.encode(prompt) == ref(prompt, add_special_tokens=False).input_ids


def test_batch_call_shape(tok_dir):
    ours = CLIPBPETokenizer.from_folder(tok_dir)
    ids = ours(["a beach", "thunder and rain"])
    assert ids.shape == (2, 77) and ids.dtype == torch.long
    assert ids[0, 0].item() == ours.bos_id and ids[0, -1].item() == ours.pad_id


def test_pipeline_tokenizer_selection(tok_dir, tmp_path):
    """A folder with tokenizer/ gets the BPE tokenizer; otherwise the offline hash ids."""
    from clap2diffusion_amd.text_encoder import make_tokenizer, prompt_to_ids
    (tmp_path / "tokenizer").mkdir()
    for f in tok_dir.iterdir():
        (tmp_path / "tokenizer" / f.name).write_bytes(f.read_bytes())
    bpe = make_tokenizer(tmp_path)
    assert isinstance(bpe, CLIPBPETokenizer)
    fallback = make_tokenizer(None)
    assert fallback(["a beach"]).tolist() == [prompt_to_ids("a beach")]
    assert make_tokenizer(tmp_path / "missing")(["a beach"]).tolist() == [prompt_to_ids("a beach")]
