import asyncio

from django.core.management import BaseCommand

from assistant.ai.services.ai_service import get_ai_embdedder
from assistant.rag.services.search_service import embeddings_similarity


class Command(BaseCommand):
    help = "Embed two texts and print their cosine similarity"

    def add_arguments(self, parser):
        parser.add_argument("query1", type=str)
        parser.add_argument("query2", type=str)
        parser.add_argument("--model", default="nomic-embed-text", type=str)

    def handle(self, *args, **options):
        emb = asyncio.run(get_ai_embdedder(options["model"]).embeddings([options["query1"], options["query2"]]))
        self.stdout.write(f"Score: {embeddings_similarity(emb[0], emb[1])}")
