/*
 * HGGpuTraversal.java -- drop-in HGTraversal (core/.../algorithms/HGTraversal.java:36-63) whose
 * next() sequence is computed on the GPU: the exact (link, atom) pairs of
 * HGBreadthFirstTraversal(start, DefaultALGenerator, maxDistance).next() in the reference's FIFO
 * order, including the link through which each atom was first discovered
 * (core/.../algorithms/HGBreadthFirstTraversal.java:49-66,143-156) -- hgx_bfs_sequence.
 *
 * Accelerated generators: DefaultALGenerator (core/.../algorithms/DefaultALGenerator.java) with
 *   linkPredicate  == null or an AtomTypeCondition (getters :517-592),
 *   siblingPredicate == null, and any of the four booleans.
 * Anything else -- another HGALGenerator, a sibling predicate, another link predicate, or an engine
 * status HGX_E_UNSUPPORTED -- runs the reference HGBreadthFirstTraversal unchanged.
 *
 * The batch form (bfsBatch) is what TraversalBasedQuery (core/.../query/impl/TraversalBasedQuery.java:
 * 47-71) and the subsumption translators (core/.../query/cond2qry/ToQueryMap.java:282-370) need: the
 * per-depth visited sets of many start atoms at once (hgx_bfs_batch).
 *
 * UNVERIFIED: written against the cited reference interfaces; no JDK exists in this build image.
 */
package org.hypergraphdb.gpu;

import java.util.ArrayList;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import org.hypergraphdb.HGHandle;
import org.hypergraphdb.HyperGraph;
import org.hypergraphdb.algorithms.DefaultALGenerator;
import org.hypergraphdb.algorithms.HGALGenerator;
import org.hypergraphdb.algorithms.HGBreadthFirstTraversal;
import org.hypergraphdb.algorithms.HGTraversal;
import org.hypergraphdb.HGQuery.hg;
import org.hypergraphdb.query.AtomTypeCondition;
import org.hypergraphdb.util.Pair;
import org.hypergraphdb.util.Ref;

public class HGGpuTraversal implements HGTraversal
{
    private final HGGpuSnapshot snap;
    private final Ref<HGHandle> startRef;
    private HGHandle start;
    private final HGALGenerator gen;
    private final int maxDistance;
    private HGTraversal cpu;              // the reference traversal when the generator is not accelerated
    private int[] links, atoms;           // the next() sequence (ranks)
    private int pos;
    private final Set<HGHandle> visited = new HashSet<HGHandle>();

    public HGGpuTraversal(HGGpuSnapshot snap, HGHandle start, HGALGenerator gen)
    {
        this(snap, start, gen, Integer.MAX_VALUE);
    }

    public HGGpuTraversal(HGGpuSnapshot snap, HGHandle start, HGALGenerator gen, int maxDistance)
    {
        this(snap, hg.constant(start), gen, maxDistance);
    }

    public HGGpuTraversal(HGGpuSnapshot snap, Ref<HGHandle> start, HGALGenerator gen)
    {
        this(snap, start, gen, Integer.MAX_VALUE);
    }

    /**
     * The reference resolves the start reference in its constructor (HGBreadthFirstTraversal.java:
     * 122-128 calls init(), :42-47), i.e. when ToQueryMap's translators build the query; so does this
     * class.  The GPU call itself is deferred to the first hasNext() / next() / isVisited().
     */
    public HGGpuTraversal(HGGpuSnapshot snap, Ref<HGHandle> start, HGALGenerator gen, int maxDistance)
    {
        this.snap = snap;
        this.startRef = start;
        this.start = start.get();
        this.gen = gen;
        this.maxDistance = maxDistance;
        if (options(snap, gen) == null)
            cpu = new HGBreadthFirstTraversal(start, gen, maxDistance);
    }

    /**
     * The engine options of a generator: {link type key or NO_TYPE, preceding, succeeding, reverse,
     * source}, or null when the generator is not accelerated.  An AtomTypeCondition on a type no
     * stored link has yields type key -2 (nothing matches: only the start atom is reachable).
     */
    static int[] options(HGGpuSnapshot snap, HGALGenerator g)
    {
        if (!(g instanceof DefaultALGenerator)) return null;
        DefaultALGenerator d = (DefaultALGenerator)g;
        if (d.getSiblingPredicate() != null) return null;
        int type = Hgx.NO_TYPE;
        if (d.getLinkPredicate() != null)
        {
            if (!(d.getLinkPredicate() instanceof AtomTypeCondition)) return null;
            HGHandle th = ((AtomTypeCondition)d.getLinkPredicate()).getTypeHandle(snap.getGraph());
            if (th == null) return null;
            int k = snap.typeKeyOrNone(th);
            type = k >= 0 ? k : Integer.MAX_VALUE;   // no stored link of that type: a key nothing carries
        }
        return new int[] {type, d.isReturnPreceeding() ? 1 : 0, d.isReturnSucceeding() ? 1 : 0,
                          d.isReverseOrder() ? 1 : 0, d.isReturnSource() ? 1 : 0};
    }

    /** Entries per native read of a large result (sequence columns, visited sets). */
    static final int PAGE = 1 << 24;

    private static int depth(int maxDistance) { return maxDistance == Integer.MAX_VALUE ? Hgx.UNBOUNDED : maxDistance; }

    private void init()
    {
        if (links != null || cpu != null) return;
        int[] o = options(snap, gen);
        long s;
        long ctx = snap.acquireContext();   // its own stream: traversals of other threads run alongside
        try
        {
            s = Hgx.bfsSequence(ctx, new int[] {snap.rank(start)}, depth(maxDistance), o[0], o[1] != 0,
                                o[2] != 0, o[3] != 0, o[4] != 0);
        }
        catch (UnsupportedOperationException e)
        {   // e.g. ranks appended out of handle order since the export: keep the reference traversal
            cpu = new HGBreadthFirstTraversal(start, gen, maxDistance);
            return;
        }
        finally
        {
            snap.releaseContext(ctx);   // the sequence result is host data
        }
        try
        {
            links = Hgx.seqLinks(s);
            atoms = Hgx.seqAtoms(s);
        }
        finally
        {
            Hgx.seqFree(s);
        }
        visited.add(start);   // examined.put(start, TRUE) at init (HGBreadthFirstTraversal.java:42-46)
    }

    public boolean hasNext()
    {
        init();
        if (cpu != null) return cpu.hasNext();
        return pos < atoms.length;
    }

    /** The next (link, atom) pair, or null when the traversal is exhausted (HGBreadthFirstTraversal.java:143-156). */
    public Pair<HGHandle, HGHandle> next()
    {
        init();
        if (cpu != null) return cpu.next();
        if (pos >= atoms.length) return null;
        HGHandle a = snap.handle(atoms[pos]);
        Pair<HGHandle, HGHandle> p = new Pair<HGHandle, HGHandle>(snap.handle(links[pos]), a);
        pos++;
        visited.add(a);   // visited once returned (HGTraversal.isVisited contract)
        return p;
    }

    public boolean isVisited(HGHandle handle)
    {
        init();
        if (cpu != null) return cpu.isVisited(handle);
        return visited.contains(handle);
    }

    public void remove() { throw new UnsupportedOperationException(); }   // HGBreadthFirstTraversal.java:98-101

    /** Restart from the (re-resolved) start atom (HGBreadthFirstTraversal.java:158-163). */
    public void reset()
    {
        start = startRef.get();
        links = atoms = null;
        pos = 0;
        visited.clear();
        if (cpu != null)
            cpu = new HGBreadthFirstTraversal(startRef, gen, maxDistance);
    }

    /**
     * The next() atoms of many traversals at once, each in the reference's FIFO order: result[i] =
     * the atoms HGBreadthFirstTraversal(starts[i], gen, maxDistance) returns (one hgx_bfs_sequence
     * call for all starts).  Returns null when the generator is not accelerated.
     */
    public static HGHandle[][] sequences(HGGpuSnapshot snap, HGHandle[] starts, HGALGenerator gen, int maxDistance)
    {
        int[] o = options(snap, gen);
        if (o == null) return null;
        long ctx = snap.acquireContext();   // applies pending store events: ranks after it
        long s;
        try
        {
            int[] seeds = new int[starts.length];
            for (int i = 0; i < starts.length; i++)
                seeds[i] = snap.rank(starts[i]);
            s = Hgx.bfsSequence(ctx, seeds, depth(maxDistance), o[0], o[1] != 0, o[2] != 0, o[3] != 0, o[4] != 0);
        }
        finally
        {
            snap.releaseContext(ctx);
        }
        try
        {
            // the pairs of all starts may exceed one Java array (2^31): read each start's atoms by pages
            // of the flattened sequence (seqRange), never the whole column at once
            long[] off = Hgx.seqOffsets(s);
            HGHandle[][] out = new HGHandle[starts.length][];
            for (int i = 0; i < starts.length; i++)
            {
                HGHandle[] row = new HGHandle[(int)(off[i + 1] - off[i])];   // one traversal <= num_atoms < 2^31
                for (int k = 0; k < row.length; )
                {
                    int[] page = Hgx.seqRange(s, 1, off[i] + k, Math.min(row.length - k, PAGE));
                    for (int a : page)
                        row[k++] = snap.handle(a);   // FIFO order: no re-sort
                }
                out[i] = row;
            }
            return out;
        }
        finally
        {
            Hgx.seqFree(s);
        }
    }

    /**
     * Per-depth visited sets of many traversals at once: result[i][d] = the atoms the traversal
     * from starts[i] returns at distance d (result[i][0] = {starts[i]}), each in handle order.
     * Returns null when the generator is not accelerated (the caller keeps the reference path).
     */
    public static List<HGHandle[][]> bfsBatch(HGGpuSnapshot snap, HGHandle[] starts, HGALGenerator gen,
                                              int maxDistance)
    {
        int[] o = options(snap, gen);
        if (o == null) return null;
        long ctx = snap.acquireContext();   // applies pending store events: ranks after it
        long r;
        try
        {
            int[] seeds = new int[starts.length];
            for (int i = 0; i < starts.length; i++)
                seeds[i] = snap.rank(starts[i]);
            r = Hgx.bfsBatch(ctx, seeds, depth(maxDistance), o[0], o[1] != 0, o[2] != 0, o[3] != 0, o[4] != 0);
        }
        catch (RuntimeException e)
        {
            snap.releaseContext(ctx);
            throw e;
        }
        try
        {
            int levels = Hgx.bfsInfo(r)[1];
            List<HGHandle[][]> out = new ArrayList<HGHandle[][]>(starts.length);
            for (int i = 0; i < starts.length; i++)
            {
                HGHandle[][] byDepth = new HGHandle[levels][];
                for (int d = 0; d < levels; d++)
                {
                    // paged: the first page also reports nothing about the total, so read until short
                    List<HGHandle> set = new ArrayList<HGHandle>();
                    for (long first = 0; ; first += PAGE)
                    {
                        int[] page = Hgx.bfsVisitedRange(r, i, d, first, PAGE);
                        for (HGHandle h : snap.handles(page)) set.add(h);
                        if (page.length < PAGE) break;
                    }
                    byDepth[d] = set.toArray(new HGHandle[set.size()]);
                }
                out.add(byDepth);
            }
            return out;
        }
        finally
        {
            Hgx.bfsFree(r);
            snap.releaseContext(ctx);
        }
    }
}
