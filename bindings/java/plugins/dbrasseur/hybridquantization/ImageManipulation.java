package plugins.dbrasseur.hybridquantization;

/**
 * Drop-in replacement of the plugin's JavaCL backend (reference
 * src/plugins/dbrasseur/hybridquantization/ImageManipulation.java, "IM") on
 * libhq, the MI355X HIP evaluator, through the JNI shim bindings/jni/hq_jni.c.
 *
 * The public surface is the one HybridQuantization (HQ) and ScielabProcessor
 * (SP) call -- constructor (IM:52), RGBtoXYZ (IM:100), XYZtoScielab (IM:285),
 * findBestQuantization (IM:383), quantize (IM:770), updateOpenCLFilters
 * (IM:800), computeError (IM:858), close (IM:265), getOpenCLAvailable (IM:95) --
 * so HQ, SP and SWASA compile unchanged against it.  The simulated-annealing
 * policy stays in Java (SWASA, with icy.util.Random as in the reference); only
 * the per-population candidate cost (IM:620-727) runs natively.
 *
 * Without libhq_jni or a GPU the class behaves like the reference without
 * OpenCL (IM:79-92): the constructor prints a warning, updateOpenCLFilters only
 * stores the packed filters, RGBtoXYZ takes the reference's Java path
 * (IM:139-149), XYZtoScielab / findBestQuantization / quantize return zero
 * arrays (IM:369, IM:590, IM:797).  computeError needs the GPU (the reference
 * has no fallback there either, IM:858-894).
 *
 * This file has not been compiled: the build image has no JDK (INTEGRATION.md).
 */
public class ImageManipulation {
    public enum deltaETypes {CIE76, CIE94, CIEDE2000}

    private static final boolean NATIVE_LOADED;

    static {
        boolean ok;
        try {
            System.loadLibrary("hq_jni"); // libhq_jni.so next to libhq.so on java.library.path
            ok = true;
        } catch (UnsatisfiedLinkError e) {
            ok = false;
        }
        NATIVE_LOADED = ok;
    }

    private long ctx;
    private boolean openCLAvailable; // name kept: HQ/SP read it through getOpenCLAvailable()
    private boolean filtersReady;
    private final boolean verbose;
    private final boolean convergence;

    public ImageManipulation(deltaETypes deltaEType, boolean verbose, boolean convergence) {
        this.verbose = verbose;
        this.convergence = convergence;
        this.ctx = NATIVE_LOADED ? nCreate(0, deltaEType.ordinal()) : 0L;
        this.openCLAvailable = ctx != 0L;
        if (!openCLAvailable)
            System.out.println("Warning (HybridQuantization): no MI355X/HIP device or libhq_jni; GPU path unavailable.");
    }

    boolean getOpenCLAvailable() {
        return openCLAvailable;
    }

    private void require() {
        if (!openCLAvailable) throw new IllegalStateException("libhq: no usable GPU (see constructor warning)");
    }

    public float[] RGBtoXYZ(float[] R, float[] G, float[] B) {
        float[] out = new float[4 * R.length];
        if (openCLAvailable) {
            nRGBtoXYZ(ctx, R, G, B, out);
            return out;
        }
        for (int i = 0; i < R.length; i++) { // IM:139-149 Java mode
            float[] xyz = ScielabProcessor.sRGBtoXYZ(new float[]{R[i], G[i], B[i]});
            int off = i << 2;
            out[off] = xyz[0];
            out[off + 1] = xyz[1];
            out[off + 2] = xyz[2];
            out[off + 3] = 0.0f;
        }
        return out;
    }

    public float[] XYZtoScielab(float[] XYZ, float[][][] filters, float[] absfilters, int w, float[] illuminant) {
        float[] lab = new float[XYZ.length];
        if (!openCLAvailable) return lab; // IM:369
        if (!filtersReady) updateOpenCLFilters(filters, absfilters);
        nXYZtoScielab(ctx, XYZ, w, illuminant, lab);
        return lab;
    }

    private int taps;
    private float[] k1, k2, k3, absk3;

    /** Packs Ofilters[3][][] into k1/k2 (float4 taps) and k3/|k3| like IM:800-841;
     *  uploads them when the GPU is there (SP:180 calls this unconditionally). */
    public void updateOpenCLFilters(float[][][] filters, float[] absfilters) {
        taps = filters[0][0].length;
        k1 = new float[4 * taps];
        k2 = new float[4 * taps];
        for (int t = 0; t < taps; t++) {
            for (int c = 0; c < 3; c++) {
                k1[4 * t + c] = filters[c][0][t];
                k2[4 * t + c] = filters[c][1][t];
            }
        }
        k3 = filters[0][2].clone();
        absk3 = absfilters.clone();
        if (openCLAvailable) nSetFilters(ctx, taps, k1, k2, k3, absk3);
        filtersReady = true;
    }

    /** IM:383-591: same SA loop and SWASA calls as the reference; costs from the GPU. */
    public float[] findBestQuantization(float[] rgb, float[] lab, int w, int K, SWASA sa,
                                        float[][][] filters, float[] absfilters, float[] illuminant) {
        sa.reset();
        float[] best = new float[4 * K];
        double bestError = 0;
        if (openCLAvailable) {
            if (!filtersReady) updateOpenCLFilters(filters, absfilters);
            nSetImage(ctx, rgb, lab, w, illuminant);
            int P = sa.getPopulationSize();
            float[][] colors = new float[P][];
            for (int i = 0; i < P; i++) colors[i] = sa.generateRandomColors(K);
            float[][] candidate = new float[P][4 * K];
            double[] current = evalPopulation(colors, K, sa);
            int m = argmin(current);
            bestError = current[m];
            System.arraycopy(colors[m], 0, best, 0, best.length);
            int imax = sa.getImax();
            for (int ite = 1; ite <= imax; ite++) {
                if (sa.getPlugin() != null && sa.getPlugin().isStopFlag()) break;
                sa.reduceTemperatureIfNecessary(ite);
                for (int j = 0; j < P; j++) sa.generateNeighboringColors(colors[j], candidate[j], K, ite);
                double[] errors = evalPopulation(candidate, K, sa);
                double minError = Double.MAX_VALUE;
                int minIdx = 0;
                for (int i = 0; i < P; i++) {
                    if (P > 1 && errors[i] < minError) { minError = errors[i]; minIdx = i; }
                    if (sa.isAccepted(errors[i] - current[i])) {
                        current[i] = errors[i];
                        System.arraycopy(candidate[i], 0, colors[i], 0, candidate[i].length);
                        if (current[i] < bestError) {
                            bestError = current[i];
                            System.arraycopy(candidate[i], 0, best, 0, best.length);
                            if (verbose) System.out.println("Best Error :" + bestError);
                        }
                    }
                }
                for (int i = 0; convergence && P > 1 && i < P; i++) {
                    if (!sa.keepsHisValues(ite)) {
                        current[i] = minError;
                        System.arraycopy(candidate[minIdx], 0, colors[i], 0, candidate[minIdx].length);
                    }
                }
                if (ite % 10 == 0 && sa.getPlugin() != null)
                    sa.getPlugin().updateProgressBar(ite + "/" + imax, (ite * 1.0) / imax);
            }
        }
        System.out.printf("Final error : %.5f\n", bestError);
        return best;
    }

    /** IM:620-727 on the GPU: mean dE per palette + SWASA penalty (IM:712). */
    private double[] evalPopulation(float[][] palettes, int K, SWASA sa) {
        int P = palettes.length;
        float[] flat = new float[P * 4 * K];
        for (int p = 0; p < P; p++) System.arraycopy(palettes[p], 0, flat, p * 4 * K, 4 * K);
        double[] mean = new double[P];
        int[] used = new int[P * K];
        nEvalPopulation(ctx, flat, P, K, mean, used);
        double[] cost = new double[P];
        int[] u = new int[K];
        for (int p = 0; p < P; p++) {
            System.arraycopy(used, p * K, u, 0, K);
            cost[p] = mean[p] + sa.computePenalty(u);
        }
        return cost;
    }

    public float[] quantize(float[] inlineImageRGB, float[] colors) {
        float[] out = new float[inlineImageRGB.length];
        if (openCLAvailable) nQuantize(ctx, inlineImageRGB, colors, out);
        return out;
    }

    public double computeError(float[] original, float[] quantized, float[] errorImage) {
        require();
        return nComputeError(ctx, original, quantized, errorImage);
    }

    public void close() {
        if (ctx != 0L) nDestroy(ctx);
        ctx = 0L;
        openCLAvailable = false;
    }

    public static int argmin(double[] arr) {
        int min = 0;
        for (int i = 1; i < arr.length; i++) if (arr[min] > arr[i]) min = i;
        return min;
    }

    private static native long nCreate(int device, int deType);
    private static native void nDestroy(long ctx);
    private static native void nSetFilters(long ctx, int taps, float[] k1, float[] k2, float[] k3, float[] absk3);
    private static native void nRGBtoXYZ(long ctx, float[] R, float[] G, float[] B, float[] out);
    private static native void nXYZtoScielab(long ctx, float[] xyz, int w, float[] illum, float[] out);
    private static native void nSetImage(long ctx, float[] rgba, float[] lab, int w, float[] illum);
    private static native void nEvalPopulation(long ctx, float[] palettes, int P, int K, double[] mean, int[] used);
    private static native void nQuantize(long ctx, float[] rgba, float[] colors, float[] out);
    private static native double nComputeError(long ctx, float[] orig, float[] quant, float[] errImg);
}
