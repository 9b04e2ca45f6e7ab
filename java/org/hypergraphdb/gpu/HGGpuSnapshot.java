/*
 * HGGpuSnapshot.java -- the device snapshot of one HyperGraph: export from the store, the .hgcsr
 * file, rank <-> handle maps and incremental refresh from store events (SURVEY.md 8(f) rank 1).
 *
 *   export:  every atom handle via hg.all() = AnyAtomCondition -> IndexScanQuery(indexByType)
 *            (core/.../query/cond2qry/ToQueryMap.java:101-113); handles ranked in unsigned byte
 *            order (the BJE comparator, storage/bdb-je/.../BJEStorageImplementation.java:109-111;
 *            UUID.compareTo, core/.../handle/UUID.java:364-376); every layout [type, value,
 *            t0..tk-1] read with HGStore.getLink (core/.../HGStore.java:179-191; written at
 *            HyperGraph.java:1603-1608) -> hgx_graph_create (include/hgx.h).
 *   refresh: an HGListener for HGAtomAddedEvent / HGAtomRemovedEvent / HGAtomReplacedEvent
 *            (core/.../event/) queues link changes; sync() applies them in ONE hgx_graph_update
 *            (a replace = remove + add of the same atom in one batch).  New atoms take ranks after
 *            the existing ones; when one of them sorts before an existing handle (random UUIDs),
 *            result sets are re-sorted by handle here and the order-exact traversal is refused by
 *            the engine (HGX_OPT_RANKS_ORDERED) until the next export.
 *
 * UNVERIFIED: written against the cited reference interfaces; no JDK exists in this build image.
 */
package org.hypergraphdb.gpu;

import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.Comparator;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import org.hypergraphdb.HGException;
import org.hypergraphdb.HGHandle;
import org.hypergraphdb.HGPersistentHandle;
import org.hypergraphdb.HGQuery.hg;
import org.hypergraphdb.HGSearchResult;
import org.hypergraphdb.HyperGraph;
import org.hypergraphdb.event.HGAtomAddedEvent;
import org.hypergraphdb.event.HGAtomRemovedEvent;
import org.hypergraphdb.event.HGAtomReplacedEvent;
import org.hypergraphdb.event.HGEvent;
import org.hypergraphdb.event.HGListener;

public final class HGGpuSnapshot implements AutoCloseable
{
    /** Unsigned lexicographic order of persistent-handle bytes (UUID.java:364-376, BAUtils.java:55-80). */
    public static final Comparator<HGPersistentHandle> HANDLE_ORDER = new Comparator<HGPersistentHandle>() {
        public int compare(HGPersistentHandle a, HGPersistentHandle b) { return compareBytes(a.toByteArray(), b.toByteArray()); }
    };

    static int compareBytes(byte[] x, byte[] y)
    {
        int n = Math.min(x.length, y.length);
        for (int i = 0; i < n; i++)
        {
            int d = (x[i] & 0xff) - (y[i] & 0xff);
            if (d != 0) return d;
        }
        return x.length - y.length;
    }

    private final HyperGraph graph;
    private final int device;
    private long g;                                   // hgx_graph*
    private final List<HGPersistentHandle> byRank = new ArrayList<HGPersistentHandle>();
    private final Map<HGPersistentHandle, Integer> rankOf = new HashMap<HGPersistentHandle, Integer>();
    private final Map<HGPersistentHandle, Integer> typeKeyOf = new HashMap<HGPersistentHandle, Integer>();
    private int orderedPrefix;                        // ranks below this are in handle order
    private final List<HGPersistentHandle> pendingAdd = new ArrayList<HGPersistentHandle>();
    private final List<HGPersistentHandle> pendingRemove = new ArrayList<HGPersistentHandle>();
    private final ArrayDeque<Long> idleContexts = new ArrayDeque<Long>();   // hgx_graph_context handles
    private int busyContexts;
    private final HGListener listener = new HGListener() {
        public Result handle(HyperGraph graph, HGEvent event)
        {
            synchronized (HGGpuSnapshot.this)
            {
                if (event instanceof HGAtomAddedEvent)
                    pendingAdd.add(graph.getPersistentHandle(((HGAtomAddedEvent)event).getAtomHandle()));
                else if (event instanceof HGAtomRemovedEvent)
                    pendingRemove.add(graph.getPersistentHandle(((HGAtomRemovedEvent)event).getAtomHandle()));
                else if (event instanceof HGAtomReplacedEvent)
                {   // same handle, new type + targets: remove + add in one batch
                    HGPersistentHandle h = graph.getPersistentHandle(((HGAtomReplacedEvent)event).getAtomHandle());
                    pendingRemove.add(h);
                    pendingAdd.add(h);
                }
            }
            return Result.ok;
        }
    };

    private HGGpuSnapshot(HyperGraph graph, int device)
    {
        this.graph = graph;
        this.device = device;
    }

    /** Walk the store once and build the device snapshot on {@code device}. */
    public static HGGpuSnapshot export(HyperGraph graph, int device)
    {
        HGGpuSnapshot s = new HGGpuSnapshot(graph, device);
        List<HGPersistentHandle> all = new ArrayList<HGPersistentHandle>();
        HGSearchResult<HGHandle> rs = graph.find(hg.all());       // IndexScanQuery(indexByType)
        try
        {
            while (rs.hasNext())
                all.add(graph.getPersistentHandle(rs.next()));
        }
        finally
        {
            rs.close();
        }
        all.sort(HANDLE_ORDER);
        for (HGPersistentHandle h : all)
            s.appendRank(h);
        s.orderedPrefix = all.size();
        Rows r = s.rowsOf(all);
        s.g = Hgx.graphCreate(all.size(), r.linkAtom, r.tgtOff, r.tgtIdx, r.linkType, device);
        s.register();
        return s;
    }

    /** Map a .hgcsr file written by {@link #save} (ranks map back through its handle table). */
    public static HGGpuSnapshot open(HyperGraph graph, String path, int device)
    {
        HGGpuSnapshot s = new HGGpuSnapshot(graph, device);
        long[] info = Hgx.snapshotInfo(path);                     // {A, M, P, handle_bytes, has_types}
        int hb = (int)info[3];
        if (hb <= 0)
            throw new HGException("hgcsr file " + path + " has no handle table");
        // the handle table by ranges (a config-4 store: 300M 16-byte handles = 4.8 GB, beyond one
        // byte[]); the whole file's checksum is verified once first
        Hgx.snapshotVerify(path);
        final long A = info[0];
        final long step = Math.max(1, TABLE_CHUNK_BYTES / hb);
        for (long r0 = 0; r0 < A; r0 += step)
        {
            long n = Math.min(step, A - r0);
            byte[] table = Hgx.snapshotHandlesRange(path, r0, n);
            for (int k = 0; k < n; k++)
                s.appendRank(graph.getHandleFactory().makeHandle(table, k * hb));
        }
        s.orderedPrefix = (int)A;
        s.g = Hgx.graphOpen(path, device);
        for (int r = 0; r < s.byRank.size(); r++)                 // type keys of the stored links
        {
            HGPersistentHandle[] layout = graph.getStore().getLink(s.byRank.get(r));
            if (layout != null && layout.length > 2) s.typeKey(layout[0]);
        }
        s.register();
        return s;
    }

    /** Write the snapshot rows + rank-ordered handle table (hgx_snapshot_write, atomic replace). */
    public synchronized void save(String path)
    {
        Rows r = rowsOf(byRank);
        final int hb = byRank.isEmpty() ? 0 : byRank.get(0).toByteArray().length;
        // streamed: the rows, then the handle table in pieces of TABLE_CHUNK_BYTES (long arithmetic: the
        // table of a 300M-atom store is 4.8 GB, beyond one byte[] and beyond int byte offsets)
        long w = Hgx.snapshotWriterBegin(path, byRank.size(), r.linkAtom, r.tgtOff, r.tgtIdx, r.linkType, hb);
        boolean ended = false;   // end frees the writer whether or not it succeeds
        try
        {
            final int per = hb > 0 ? (int)Math.max(1, TABLE_CHUNK_BYTES / hb) : 0;
            for (int i0 = 0; hb > 0 && i0 < byRank.size(); i0 += per)
            {
                int n = Math.min(per, byRank.size() - i0);
                byte[] chunk = new byte[n * hb];   // n * hb <= TABLE_CHUNK_BYTES
                for (int k = 0; k < n; k++)
                    System.arraycopy(byRank.get(i0 + k).toByteArray(), 0, chunk, k * hb, hb);
                Hgx.snapshotWriterHandles(w, chunk, hb);
            }
            ended = true;
            Hgx.snapshotWriterEnd(w);
        }
        finally
        {
            if (!ended) Hgx.snapshotWriterAbort(w);   // removes the partial file
        }
    }

    /** Bytes of handle table per native read / write (well below the 2^31 limit of one byte[]). */
    static final long TABLE_CHUNK_BYTES = 1L << 28;

    private void register()
    {
        graph.getEventManager().addListener(HGAtomAddedEvent.class, listener);
        graph.getEventManager().addListener(HGAtomRemovedEvent.class, listener);
        graph.getEventManager().addListener(HGAtomReplacedEvent.class, listener);
    }

    private int appendRank(HGPersistentHandle h)
    {
        Integer r = rankOf.get(h);
        if (r != null) return r;
        rankOf.put(h, byRank.size());
        byRank.add(h);
        return byRank.size() - 1;
    }

    private int typeKey(HGPersistentHandle type)
    {
        Integer k = typeKeyOf.get(type);
        if (k == null)
        {
            k = typeKeyOf.size();
            typeKeyOf.put(type, k);
        }
        return k;
    }

    /** Dense type key of a type handle, or -1 when no stored link has that type. */
    public synchronized int typeKeyOrNone(HGHandle type)
    {
        Integer k = typeKeyOf.get(graph.getPersistentHandle(type));
        return k == null ? -1 : k;
    }

    private static final class Rows
    {
        int[] linkAtom, tgtIdx, linkType;
        long[] tgtOff;
    }

    /** Link rows of the given atoms (ascending rank): layouts with arity > 0 (HGStore.getLink). */
    private Rows rowsOf(List<HGPersistentHandle> atoms)
    {
        List<int[]> targets = new ArrayList<int[]>();
        List<Integer> la = new ArrayList<Integer>(), ty = new ArrayList<Integer>();
        long pins = 0;
        for (HGPersistentHandle h : atoms)
        {
            HGPersistentHandle[] layout = graph.getStore().getLink(h);   // [type, value, t0..tk-1]
            if (layout == null || layout.length <= 2)
                continue;   // a node (or an arity-0 link: no incidence, never an anchored result)
            int[] t = new int[layout.length - 2];
            for (int i = 2; i < layout.length; i++)
                t[i - 2] = rankOf.get(layout[i]);
            la.add(rankOf.get(h));
            ty.add(typeKey(layout[0]));
            targets.add(t);
            pins += t.length;
        }
        if (pins > Integer.MAX_VALUE - 8)   // one int[] of targets: 2^31 pins (config 4 has 1.0e9)
            throw new HGException("snapshot: " + pins + " link targets exceed one Java array; export it with "
                                  + "the native exporter (hgx_snapshot_writer_*) instead");
        Rows r = new Rows();
        r.linkAtom = new int[la.size()];
        r.linkType = new int[la.size()];
        r.tgtOff = new long[la.size() + 1];
        r.tgtIdx = new int[(int)pins];
        int p = 0;
        for (int i = 0; i < la.size(); i++)
        {
            r.linkAtom[i] = la.get(i);
            r.linkType[i] = ty.get(i);
            for (int t : targets.get(i)) r.tgtIdx[p++] = t;
            r.tgtOff[i + 1] = p;
        }
        return r;
    }

    /**
     * Apply the queued store events to the device snapshot (one hgx_graph_update).  Called by the
     * GPU query / traversal classes before they run; safe to call from any thread.
     */
    public synchronized void sync()
    {
        if (pendingAdd.isEmpty() && pendingRemove.isEmpty()) return;
        while (busyContexts > 0)   // hgx_graph_update is refused while an execution context exists
        {
            try { wait(); }
            catch (InterruptedException e)
            {
                Thread.currentThread().interrupt();
                throw new HGException("interrupted while GPU traversals finish", e);
            }
        }
        dropIdleContexts();
        int before = byRank.size();
        HGPersistentHandle maxOld = before > 0 ? byRank.get(orderedPrefix - 1) : null;
        boolean ordered = true;
        int[] rm = new int[pendingRemove.size()];
        int nrm = 0;
        for (HGPersistentHandle h : pendingRemove)
        {
            Integer r = rankOf.get(h);
            if (r != null) rm[nrm++] = r;                          // removing an unknown atom: no-op
        }
        List<HGPersistentHandle> adds = new ArrayList<HGPersistentHandle>();
        for (HGPersistentHandle h : pendingAdd)
        {
            if (!rankOf.containsKey(h))
            {
                if (maxOld != null && HANDLE_ORDER.compare(h, maxOld) < 0) ordered = false;
                appendRank(h);                                     // ranks after the existing ones
            }
            adds.add(h);
        }
        Rows r = rowsOf(adds);                                      // links only; nodes just grow the space
        Hgx.graphUpdate(g, byRank.size(), r.linkAtom, r.tgtOff, r.tgtIdx, r.linkType, Arrays.copyOf(rm, nrm));
        if (ordered && byRank.size() > before)
        {   // appended handles all sort after the old ones (IntHandleFactory): rank order == handle order
            orderedPrefix = byRank.size();
            Hgx.setOption(g, Hgx.OPT_RANKS_ORDERED, 1);
        }
        pendingAdd.clear();
        pendingRemove.clear();
    }

    public synchronized int rank(HGHandle h)
    {
        Integer r = rankOf.get(graph.getPersistentHandle(h));
        if (r == null) throw new HGException("atom " + h + " is not in the GPU snapshot");
        return r;
    }

    public synchronized HGHandle handle(int rank) { return byRank.get(rank); }

    /** Handles of ascending ranks, in the reference's (handle) order. */
    public synchronized HGHandle[] handles(int[] ranks)
    {
        HGPersistentHandle[] out = new HGPersistentHandle[ranks.length];
        boolean appended = false;
        for (int i = 0; i < ranks.length; i++)
        {
            out[i] = byRank.get(ranks[i]);
            appended |= ranks[i] >= orderedPrefix;
        }
        if (appended) Arrays.sort(out, HANDLE_ORDER);   // appended ranks need not follow handle order
        return out;
    }

    /**
     * An execution context of the device snapshot for one traversal call (hgx_graph_context: the same
     * device arrays, its own stream, lock and scratch), so traversals issued by several threads run
     * side by side on the GPU instead of queueing on the snapshot's lock.  Pending store events are
     * applied first.  Give it back with releaseContext (contexts are pooled).
     */
    synchronized long acquireContext()
    {
        sync();
        busyContexts++;
        Long c = idleContexts.poll();
        if (c != null) return c;
        try { return Hgx.graphContext(g); }
        catch (RuntimeException e) { busyContexts--; notifyAll(); throw e; }
    }

    synchronized void releaseContext(long c)
    {
        busyContexts--;
        idleContexts.push(c);
        notifyAll();
    }

    private void dropIdleContexts()
    {
        for (Long c : idleContexts) Hgx.graphDestroy(c);
        idleContexts.clear();
    }

    public HyperGraph getGraph() { return graph; }
    public int getDevice() { return device; }
    long native_() { return g; }

    public synchronized void close()
    {
        if (g != 0)
        {
            graph.getEventManager().removeListener(HGAtomAddedEvent.class, listener);
            graph.getEventManager().removeListener(HGAtomRemovedEvent.class, listener);
            graph.getEventManager().removeListener(HGAtomReplacedEvent.class, listener);
            dropIdleContexts();   // a context still in use keeps the device snapshot alive until released
            Hgx.graphDestroy(g);
            g = 0;
        }
    }
}
